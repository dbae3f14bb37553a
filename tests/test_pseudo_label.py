"""Host logic of the data-parallel pseudo-labelling loop (kwhisper.pseudo_label), CPU only.

* the shard plan is pinned to accelerate's own BatchSamplerShard (the reference's sampler,
  run_pseudo_labelling.py:326-329 via accelerator.prepare);
* a world_size-2 gloo run returns exactly the single-process predictions in dataset order, with ragged
  per-rank widths (pad_across_processes) and a wrapped final round (gather_for_metrics remainder);
* the CSV is the reference's [file_id, str(ndarray)] format (run_pseudo_labelling.py:347-350).
"""
import csv
import os
import socket

import numpy as np
import pytest
import torch

from kwhisper.pseudo_label import gather_remainder, pseudo_label, shard_batches, step_model, write_transcription_csv

PAD = 50256


class _StubModel:
    """Deterministic stand-in for generate(): row i -> [i*10, i*10+1, ...] of length 2 + i % 5, right-padded
    with PAD to the batch's longest row (the HF output contract)."""

    def generate(self, feats, **kw):
        idx = feats[:, 0].long().tolist()
        T = max(2 + i % 5 for i in idx)
        out = torch.full((len(idx), T), PAD, dtype=torch.int64)
        for r, i in enumerate(idx):
            n = 2 + i % 5
            out[r, :n] = torch.arange(n) + 10 * i
        return out


def _features(idx):
    return torch.tensor(idx, dtype=torch.float32)[:, None]


@pytest.mark.parametrize("n", [1, 5, 31, 32, 33, 64, 100, 257])
@pytest.mark.parametrize("bs,world", [(4, 1), (4, 2), (32, 2), (3, 4), (32, 8)])
def test_shard_plan_matches_accelerate(n, bs, world):
    acc = pytest.importorskip("accelerate.data_loader")
    from torch.utils.data import BatchSampler, SequentialSampler

    for r in range(world):
        ref = list(acc.BatchSamplerShard(BatchSampler(SequentialSampler(range(n)), bs, False), num_processes=world,
                                         process_index=r, split_batches=False, even_batches=True))
        assert shard_batches(n, bs, world, r) == ref


@pytest.mark.parametrize("n,bs,world", [(100, 32, 4), (1768, 32, 8), (7, 3, 2), (64, 32, 2), (0, 32, 2)])
def test_gathered_rounds_cover_dataset_once(n, bs, world):
    """Concatenating every rank's step-s batch (rank order) and truncating the last round to the remainder
    yields 0..n-1 exactly once, in order."""
    plans = [shard_batches(n, bs, world, r) for r in range(world)]
    assert len({len(p) for p in plans}) <= 1  # every rank runs the same number of steps
    order = []
    steps = len(plans[0])
    rem = gather_remainder(n, bs, world)
    for s in range(steps):
        rnd = [i for r in range(world) for i in plans[r][s]]
        if s == steps - 1 and rem > 0:
            rnd = rnd[:rem]
        order += rnd
    assert order == list(range(n))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, bs, out_dir):
    import torch.distributed as dist

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        ids, preds = pseudo_label(_StubModel(), _features, n, batch_size=bs, pad_token_id=PAD)
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), ids=np.array(ids),
                 preds=np.array([p.tolist() + [-1] * (16 - len(p)) for p in preds]),
                 lens=np.array([len(p) for p in preds]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n,bs", [(13, 4), (16, 4), (3, 4)])
def test_gloo_world2_matches_single_process(tmp_path, n, bs):
    import torch.multiprocessing as mp

    mp.spawn(_worker, args=(2, _free_port(), n, bs, str(tmp_path)), nprocs=2, join=True)
    ids1, preds1 = pseudo_label(_StubModel(), _features, n, batch_size=bs, pad_token_id=PAD)
    assert ids1 == list(range(n))
    for r in range(2):
        z = np.load(tmp_path / f"r{r}.npz")
        assert z["ids"].tolist() == list(range(n)), "gathered order is dataset order on every rank"
        for i in range(n):
            row = z["preds"][i][: z["lens"][i]]
            k = 2 + i % 5
            np.testing.assert_array_equal(row[:k], np.arange(k) + 10 * i)  # the item's own tokens
            assert (row[k:] == PAD).all()  # then only padding (the round's common width)
            np.testing.assert_array_equal(preds1[i][:k], row[:k])


def test_transcription_csv_format(tmp_path):
    preds = [np.array([50258, 50266, 50360, 123]), np.array([7, PAD])]
    p = tmp_path / "train-transcription.csv"
    write_transcription_csv(str(p), ["a.flac", "b.flac"], preds)
    rows = list(csv.reader(open(p, encoding="UTF8")))
    assert rows[0] == ["file_id", "whisper_transcript"]
    assert rows[1] == ["a.flac", str(preds[0])] and rows[2] == ["b.flac", str(preds[1])]


class _StubTaskModel(_StubModel):
    """generate() whose output depends on the (language, task) prompt: row i -> tokens offset by the task."""

    OFF = {("ja", "transcribe"): 0, ("en", "translate"): 1000}

    def generate(self, feats, language=None, task=None, **kw):
        out = super().generate(feats, **kw)
        return torch.where(out == PAD, out, out + self.OFF[(language, task)])


TLT = [("transcription", "ja", "transcribe"), ("translation", "en", "translate")]


def test_multitask_columns_match_separate_runs():
    """run_pseudo_labelling_v3.py:309-321: one prediction column per (text, lang, task) triple, each equal
    to a single-task run with that prompt."""
    from kwhisper.pseudo_label import pseudo_label_multitask

    m = _StubTaskModel()
    ids, cols = pseudo_label_multitask(m, _features, 13, batch_size=4, text_lang_task=TLT, pad_token_id=PAD)
    assert ids == list(range(13)) and set(cols) == {"transcription", "translation"}
    for text, lang, task in TLT:
        ids1, preds1 = pseudo_label(m, _features, 13, batch_size=4, pad_token_id=PAD,
                                    gen_kwargs=dict(language=lang, task=task))
        assert ids1 == ids
        for a, b in zip(cols[text], preds1):
            np.testing.assert_array_equal(a, b)


def _mt_worker(rank, world, port, n, bs, out_dir):
    import torch.distributed as dist

    from kwhisper.pseudo_label import pseudo_label_multitask

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        ids, cols = pseudo_label_multitask(_StubTaskModel(), _features, n, batch_size=bs, text_lang_task=TLT,
                                           pad_token_id=PAD)
        np.savez(os.path.join(out_dir, f"mt{rank}.npz"), ids=np.array(ids),
                 **{t: np.array([p.tolist() + [-1] * (16 - len(p)) for p in c]) for t, c in cols.items()})
    finally:
        dist.destroy_process_group()


def test_multitask_gloo_world2(tmp_path):
    import torch.multiprocessing as mp

    from kwhisper.pseudo_label import pseudo_label_multitask

    n, bs = 11, 4
    mp.spawn(_mt_worker, args=(2, _free_port(), n, bs, str(tmp_path)), nprocs=2, join=True)
    _, ref = pseudo_label_multitask(_StubTaskModel(), _features, n, batch_size=bs, text_lang_task=TLT,
                                    pad_token_id=PAD)
    for r in range(2):
        z = np.load(tmp_path / f"mt{r}.npz")
        assert z["ids"].tolist() == list(range(n))
        for text, _, _ in TLT:
            for i in range(n):
                row = z[text][i][z[text][i] != -1]
                k = len(ref[text][i][ref[text][i] != PAD])
                np.testing.assert_array_equal(row[:k], ref[text][i][:k])
                assert (row[k:] == PAD).all()


@pytest.mark.parametrize("ts", [False, True])
def test_legacy_prompt_in_output(ts):
    """rows start with [sot, lang, task] (+ notimestamps), the layout
    run_data_filtering.py:230-251,279 indexes with timestamp_position = 3."""
    from kwhisper.config import LARGE_V3, generation_constants

    class M(_StubModel):
        generation_config = generation_constants(LARGE_V3)

    g = M.generation_config
    _, plain = pseudo_label(M(), _features, 6, batch_size=4, pad_token_id=PAD,
                            gen_kwargs=dict(language="ja", task="transcribe", return_timestamps=ts))
    _, leg = pseudo_label(M(), _features, 6, batch_size=4, pad_token_id=PAD, legacy_prompt_in_output=True,
                          gen_kwargs=dict(language="ja", task="transcribe", return_timestamps=ts))
    pre = [50258, 50266, 50360] + ([] if ts else [50364])
    assert [g.decoder_start_token_id, g.lang_to_id["<|ja|>"], g.task_to_id["transcribe"]] == pre[:3]
    for a, b in zip(plain, leg):
        assert b[: len(pre)].tolist() == pre
        np.testing.assert_array_equal(b[len(pre):], a)
    with pytest.raises(ValueError):
        pseudo_label(M(), _features, 2, batch_size=4, pad_token_id=PAD, legacy_prompt_in_output=True, gen_kwargs={})


def test_pad_token_id_is_required():
    """The cross-process pad is the tokenizer's pad id (run_pseudo_labelling.py:339), which the caller must
    state: no default that could silently be generation_config.pad_token_id."""
    with pytest.raises(TypeError):
        pseudo_label(_StubModel(), _features, 3, batch_size=4)


def test_transcription_arrow_column_matches_datasets(tmp_path):
    """The Arrow column equals what datasets' add_column("whisper_transcript", eval_preds) stores
    (run_pseudo_labelling.py:351), and the IPC file reads back to the same table."""
    pa = pytest.importorskip("pyarrow")
    datasets = pytest.importorskip("datasets")
    from kwhisper.pseudo_label import transcription_table, write_transcription_arrow

    preds = [np.array([50258, 50266, 50360, 123, PAD]), np.array([7, 8, 9, PAD, PAD])]
    fids = ["a.flac", "b.flac"]
    ds = datasets.Dataset.from_dict({"file_id": fids}).add_column("whisper_transcript", preds)
    t = transcription_table(fids, preds)
    assert t.column("whisper_transcript").to_pylist() == ds["whisper_transcript"][:]
    p = str(tmp_path / "labels.arrow")
    write_transcription_arrow(p, fids, preds)
    with pa.OSFile(p, "rb") as f:
        back = pa.ipc.open_stream(f).read_all()
    assert back.equals(t)


# ---- resume by round (SURVEY.md §5 checkpoint / resume) ---------------------------------------------------
class _CountingModel(_StubModel):
    def __init__(self):
        self.batches = []

    def generate(self, feats, **kw):
        self.batches.append(feats[:, 0].long().tolist())
        return super().generate(feats, **kw)


def _same(a, b):
    assert a[0] == b[0]
    assert len(a[1]) == len(b[1])
    for x, y in zip(a[1], b[1]):
        np.testing.assert_array_equal(x, y)


def test_resume_skips_checkpointed_rounds(tmp_path):
    ck = str(tmp_path / "ck")
    n, bs = 23, 4  # 6 rounds, the last one ragged
    ref = pseudo_label(_StubModel(), _features, n, batch_size=bs, pad_token_id=PAD)
    m1 = _CountingModel()
    run1 = pseudo_label(m1, _features, n, batch_size=bs, pad_token_id=PAD, checkpoint_dir=ck)
    _same(run1, ref)
    assert len(m1.batches) == 6
    assert sorted(os.listdir(ck)) == ["plan.json"] + [f"round_{i:06d}.npz" for i in range(6)]
    # a crash after round 3: rounds 4 and 5 never reached the disk
    for i in (4, 5):
        os.remove(os.path.join(ck, f"round_{i:06d}.npz"))
    m2 = _CountingModel()
    run2 = pseudo_label(m2, _features, n, batch_size=bs, pad_token_id=PAD, checkpoint_dir=ck)
    _same(run2, ref)
    assert m2.batches == [list(range(16, 20)), [20, 21, 22, 0]]  # only the missing rounds (the last wraps)
    m3 = _CountingModel()  # everything on disk: nothing is decoded
    _same(pseudo_label(m3, _features, n, batch_size=bs, pad_token_id=PAD, checkpoint_dir=ck), ref)
    assert m3.batches == []


def test_resume_refuses_another_plan(tmp_path):
    ck = str(tmp_path / "ck")
    pseudo_label(_StubModel(), _features, 10, batch_size=4, pad_token_id=PAD, checkpoint_dir=ck)
    with pytest.raises(ValueError, match="another plan"):
        pseudo_label(_StubModel(), _features, 10, batch_size=3, pad_token_id=PAD, checkpoint_dir=ck)


@pytest.mark.parametrize("change", ["gen_kwargs", "pad", "model"])
def test_resume_refuses_another_configuration(tmp_path, change):
    """Same items / batch / world but other generate kwargs, pad id or model (compute dtype): the old rounds
    hold other labels, so the rerun refuses them instead of mixing two configurations."""
    ck = str(tmp_path / "ck")
    kw = dict(gen_kwargs={"language": "ja", "task": "transcribe", "return_timestamps": True})
    pseudo_label(_StubModel(), _features, 10, batch_size=4, pad_token_id=PAD, checkpoint_dir=ck, **kw)
    if change == "gen_kwargs":
        kw2 = dict(gen_kwargs={"language": "ja", "task": "transcribe", "return_timestamps": False}, pad_token_id=PAD)
    elif change == "pad":
        kw2 = dict(kw, pad_token_id=PAD + 1)
    else:
        kw2 = dict(kw, pad_token_id=PAD)
    other = type("_StubBF16", (_StubModel,), {"dtype": "torch.bfloat16"}) if change == "model" else _StubModel
    with pytest.raises(ValueError, match="another plan"):
        pseudo_label(other(), _features, 10, batch_size=4, checkpoint_dir=ck, **kw2)
    pseudo_label(_StubModel(), _features, 10, batch_size=4, pad_token_id=PAD, checkpoint_dir=ck, **kw)  # same: ok


def _resume_worker(rank, world, port, n, bs, ck, out_dir, tag):
    import torch.distributed as dist

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        m = _CountingModel()
        ids, preds = pseudo_label(m, _features, n, batch_size=bs, pad_token_id=PAD, checkpoint_dir=ck)
        np.savez(os.path.join(out_dir, f"{tag}{rank}.npz"), ids=np.array(ids),
                 preds=np.array([p.tolist() + [-1] * (16 - len(p)) for p in preds]),
                 decoded=np.array([i for b in m.batches for i in b] or [-1]))
    finally:
        dist.destroy_process_group()


def test_resume_gloo_world2(tmp_path):
    import torch.multiprocessing as mp

    n, bs = 13, 2  # rounds of 2 x 2 items: 4 rounds, the last one wrapped
    ck = str(tmp_path / "ck")
    mp.spawn(_resume_worker, args=(2, _free_port(), n, bs, ck, str(tmp_path), "a"), nprocs=2, join=True)
    os.remove(os.path.join(ck, "round_000002.npz"))
    mp.spawn(_resume_worker, args=(2, _free_port(), n, bs, ck, str(tmp_path), "b"), nprocs=2, join=True)
    for r in range(2):
        a, b = np.load(tmp_path / f"a{r}.npz"), np.load(tmp_path / f"b{r}.npz")
        assert a["ids"].tolist() == b["ids"].tolist() == list(range(n))
        np.testing.assert_array_equal(a["preds"], b["preds"])
        # the second run decoded round 2 only: items 8-9 on rank 0, 10-11 on rank 1
        assert b["decoded"].tolist() == [[8, 9], [10, 11]][r]


# ---- deferred gather (gather="end": one exchange after the last batch) --------------------
def _deferred_worker(rank, world, port, n, bs, out_dir, ck):
    import torch.distributed as dist

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        m = _CountingModel()
        ids_r, preds_r = pseudo_label(_StubModel(), _features, n, batch_size=bs, pad_token_id=PAD)
        ids_e, preds_e = pseudo_label(m, _features, n, batch_size=bs, pad_token_id=PAD, gather="end",
                                      checkpoint_dir=ck or None)
        np.savez(os.path.join(out_dir, f"d{rank}.npz"), ids_r=np.array(ids_r), ids_e=np.array(ids_e),
                 pr=np.array([p.tolist() + [-1] * (16 - len(p)) for p in preds_r]),
                 pe=np.array([p.tolist() + [-1] * (16 - len(p)) for p in preds_e]),
                 decoded=np.array([i for b in m.batches for i in b] or [-1]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n,bs,world", [(13, 4, 2), (16, 4, 2), (3, 4, 2), (23, 3, 3), (0, 4, 2)])
def test_deferred_gather_equals_per_round_gather(tmp_path, n, bs, world):
    """gather="end" returns, on every rank, exactly what the reference's per-batch pad + gather returns: the same
    items in dataset order, each row padded to its round's widest rank (ragged widths, wrapped final round)."""
    import torch.multiprocessing as mp

    mp.spawn(_deferred_worker, args=(world, _free_port(), n, bs, str(tmp_path), ""), nprocs=world, join=True)
    ids1, preds1 = pseudo_label(_StubModel(), _features, n, batch_size=bs, pad_token_id=PAD, gather="end")
    assert ids1 == list(range(n))
    for r in range(world):
        z = np.load(tmp_path / f"d{r}.npz")
        if n == 0:
            continue
        assert z["ids_e"].tolist() == z["ids_r"].tolist() == list(range(n))
        np.testing.assert_array_equal(z["pe"], z["pr"])


def test_deferred_gather_single_process_equals_round():
    a = pseudo_label(_StubModel(), _features, 23, batch_size=4, pad_token_id=PAD)
    b = pseudo_label(_StubModel(), _features, 23, batch_size=4, pad_token_id=PAD, gather="end")
    _same(a, b)
    with pytest.raises(ValueError, match="gather"):
        pseudo_label(_StubModel(), _features, 3, batch_size=4, pad_token_id=PAD, gather="never")


def test_deferred_gather_resume_gloo_world2(tmp_path):
    """Deferred mode checkpoints each rank's batches itself; after one rank's file of round 2 is lost, the rerun
    decodes round 2 on both ranks (a round is done only when every rank's file of it exists) and nothing else."""
    import torch.multiprocessing as mp

    n, bs = 13, 2
    ck = str(tmp_path / "ck")
    mp.spawn(_deferred_worker, args=(2, _free_port(), n, bs, str(tmp_path), ck), nprocs=2, join=True)
    a = [np.load(tmp_path / f"d{r}.npz") for r in range(2)]
    assert sorted(f for f in os.listdir(ck) if f.endswith(".npz")) == [
        f"round_{s:06d}_rank{r:03d}.npz" for s in range(4) for r in range(2)]
    os.remove(os.path.join(ck, "round_000002_rank001.npz"))
    mp.spawn(_deferred_worker, args=(2, _free_port(), n, bs, str(tmp_path), ck), nprocs=2, join=True)
    for r in range(2):
        b = np.load(tmp_path / f"d{r}.npz")
        np.testing.assert_array_equal(a[r]["pe"], b["pe"])
        assert b["ids_e"].tolist() == list(range(n))
        assert b["decoded"].tolist() == [[8, 9], [10, 11]][r]


def test_resume_refuses_legacy_plan_unless_allowed(tmp_path):
    """A checkpoint directory written before plan.json carried config_sha256 cannot prove its rounds were decoded
    with this run's generate kwargs and weights: refused by default, resumed (with a warning) only with
    allow_legacy_checkpoint=True."""
    import json

    ck = tmp_path / "ck"
    ref = pseudo_label(_StubModel(), _features, 10, batch_size=4, pad_token_id=PAD, checkpoint_dir=str(ck))
    plan = json.loads((ck / "plan.json").read_text())
    plan.pop("config_sha256")
    (ck / "plan.json").write_text(json.dumps(plan))
    m = _CountingModel()
    with pytest.raises(ValueError, match="allow_legacy_checkpoint"):
        pseudo_label(m, _features, 10, batch_size=4, pad_token_id=PAD, checkpoint_dir=str(ck))
    with pytest.warns(RuntimeWarning, match="predates"):
        got = pseudo_label(m, _features, 10, batch_size=4, pad_token_id=PAD, checkpoint_dir=str(ck),
                           allow_legacy_checkpoint=True)
    _same(got, ref)
    assert m.batches == []


class _LaneStub(_CountingModel):
    """A stub with lane(): each lane records its own batches (the engine lanes share weights, not sessions)."""

    def __init__(self, lanes=None):
        super().__init__()
        self.lanes = lanes if lanes is not None else [self]

    def lane(self):
        other = _LaneStub(self.lanes)
        self.lanes.append(other)
        return other


@pytest.mark.parametrize("n,bs,lanes", [(23, 4, 2), (23, 4, 3), (5, 4, 2), (0, 4, 2)])
def test_lanes_return_the_single_lane_predictions(n, bs, lanes):
    """lanes > 1 (gather="end"): batches decode on several model handles from several host threads; the predictions
    (and their order) equal the single-lane run's, and every batch is decoded exactly once."""
    ref = pseudo_label(_StubModel(), _features, n, batch_size=bs, pad_token_id=PAD, gather="end")
    m = _LaneStub()
    seen = {}  # step -> the handle step_model() names inside on_step (bench_configs reads that lane's stats)

    def on_step(si, total):
        seen[si] = step_model()

    got = pseudo_label(m, _features, n, batch_size=bs, pad_token_id=PAD, gather="end", lanes=lanes, on_step=on_step)
    _same(got, ref)
    decoded = sorted(i for lane in m.lanes for b in lane.batches for i in b)
    want = sorted(i for b in shard_batches(n, bs, 1, 0) for i in b)
    assert decoded == want and len(m.lanes) == lanes
    steps = shard_batches(n, bs, 1, 0)
    assert sorted(seen) == list(range(len(steps)))
    for si, h in seen.items():  # the handle that reported step si decoded its batch
        assert list(steps[si]) in [list(b) for b in h.batches]
    with pytest.raises(ValueError, match="gather"):
        pseudo_label(_LaneStub(), _features, 3, batch_size=4, pad_token_id=PAD, lanes=2)


def test_lanes_checkpoint_resume(tmp_path):
    """lanes=2 with checkpoint_dir: the lane threads write each step's per-rank file; a rerun (any lane count)
    decodes nothing and returns the same predictions; a partial directory resumes only the missing steps."""
    ck = tmp_path / "ck"
    ref = pseudo_label(_StubModel(), _features, 23, batch_size=4, pad_token_id=PAD, gather="end")
    m = _LaneStub()
    got = pseudo_label(m, _features, 23, batch_size=4, pad_token_id=PAD, gather="end", lanes=2, checkpoint_dir=str(ck))
    _same(got, ref)
    m2 = _LaneStub()
    again = pseudo_label(m2, _features, 23, batch_size=4, pad_token_id=PAD, gather="end", lanes=3,
                         checkpoint_dir=str(ck))
    _same(again, ref)
    assert sum(len(h.batches) for h in m2.lanes) == 0
    victims = sorted(ck.glob("round_*_rank0.npz"))[1::2]
    for v in victims:
        v.unlink()
    m3 = _LaneStub()
    part = pseudo_label(m3, _features, 23, batch_size=4, pad_token_id=PAD, gather="end", lanes=2,
                        checkpoint_dir=str(ck))
    _same(part, ref)
    assert sum(len(h.batches) for h in m3.lanes) == len(victims)


# ---- dynamic batch assignment (schedule="dynamic": list scheduling over a shared counter) -----
class _SlowModel(_CountingModel):
    """Batches holding an item of ``slow`` take ``delay`` seconds (a batch with extra seek passes); ``"first"`` in
    ``slow`` makes the model's first batch slow, whichever batch its rank claimed first."""

    def __init__(self, slow=(), delay=0.0, wait_for=None, report=None, announce=None):
        super().__init__()
        self.first = "first" in slow
        self.slow, self.delay = {s for s in slow if s != "first"}, delay
        self.calls = 0
        self.wait_for, self.report = wait_for, report  # (path, count): first call blocks until path holds >= count
        self.announce = announce  # a file the first call writes "1" into before anything else

    def generate(self, feats, **kw):
        import time

        self.calls += 1
        if self.announce is not None and self.calls == 1:
            with open(self.announce + ".tmp", "w") as f:
                f.write("1")
            os.replace(self.announce + ".tmp", self.announce)
        if self.wait_for is not None and self.calls == 1:
            path, count = self.wait_for
            t_end = time.time() + 60.0  # bounded: a failure, not a hang
            while time.time() < t_end:
                try:
                    if int(open(path).read() or 0) >= count:
                        break
                except (OSError, ValueError):
                    pass
                time.sleep(0.01)
        elif (self.first and self.calls == 1) or self.slow & set(feats[:, 0].long().tolist()):
            time.sleep(self.delay)
        out = super().generate(feats, **kw)
        if self.report is not None:
            tmp = self.report + ".tmp"
            with open(tmp, "w") as f:
                f.write(str(self.calls))
            os.replace(tmp, self.report)
        return out


def _dynamic_worker(rank, world, port, n, bs, out_dir, ck, slow, lanes):
    import json

    import torch.distributed as dist

    from kwhisper.pseudo_label import last_schedule

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        ref = pseudo_label(_StubModel(), _features, n, batch_size=bs, pad_token_id=PAD)  # per-round, static
        if "blocked" in slow:  # rank 0's first batch waits until rank 1 has decoded all the others
            n_batches = len(shard_batches(n, bs, world, 0)) * world
            peer, started = os.path.join(out_dir, "rank1_calls"), os.path.join(out_dir, "rank0_started")
            # (rank 1's first batch waits until rank 0 holds one: otherwise a late rank 0 finds no batch left)
            m = (_SlowModel(wait_for=(peer, n_batches - 1), announce=started) if rank == 0
                 else _SlowModel(report=peer, wait_for=(started, 1)))
        else:
            m = _SlowModel(slow if rank == 0 else (), 0.4)
        if lanes > 1:
            m = _LaneStub()
        got = pseudo_label(m, _features, n, batch_size=bs, pad_token_id=PAD, gather="end", schedule="dynamic",
                           checkpoint_dir=ck or None, lanes=lanes)
        handles = m.lanes if lanes > 1 else [m]
        with open(os.path.join(out_dir, f"y{rank}.json"), "w") as f:
            json.dump({"same": got[0] == ref[0] and len(got[1]) == len(ref[1])
                       and all(np.array_equal(a, b) for a, b in zip(got[1], ref[1])),
                       "decoded": [b for h in handles for b in h.batches], "schedule": last_schedule()}, f)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n,bs,world,lanes", [(13, 2, 2, 1), (23, 3, 3, 1), (40, 4, 2, 2), (3, 4, 2, 1)])
def test_dynamic_schedule_gloo_equals_static(tmp_path, n, bs, world, lanes):
    """schedule="dynamic" under gloo world 2 / 3 (and with two lanes per rank): every rank returns exactly the
    reference's per-round gather (items, order, each row padded to its round's widest batch, wrapped duplicates
    dropped); every batch of the static plan is decoded exactly once, by the rank last_schedule() names."""
    import json

    import torch.multiprocessing as mp

    mp.spawn(_dynamic_worker, args=(world, _free_port(), n, bs, str(tmp_path), "", (), lanes), nprocs=world,
             join=True)
    want = {tuple(b) for r in range(world) for b in shard_batches(n, bs, world, r)}
    runs = [json.load(open(tmp_path / f"y{r}.json")) for r in range(world)]
    decoded = [tuple(b) for z in runs for b in z["decoded"]]
    assert all(z["same"] for z in runs)
    assert sorted(decoded) == sorted(want) and len(decoded) == len(want)
    plans = [shard_batches(n, bs, world, r) for r in range(world)]
    for z in runs:
        assert z["schedule"] == runs[0]["schedule"]
        for j, r in enumerate(z["schedule"]):  # global batch j = round j // W, rank slot j % W
            assert plans[j % world][j // world] in runs[r]["decoded"]


def test_dynamic_schedule_balances_a_slow_rank(tmp_path):
    """Rank 0's first batch is slow -- it does not return until rank 1 has decoded every other batch (a file rank 1's
    model rewrites after each batch; ADVICE r05: an ordering, not a sleep, so a slow process start cannot change the
    outcome): under the static plan rank 0 would still own half of the batches; with dynamic claims rank 1 decodes
    all the batches rank 0 is not ready for, and the outputs are the reference's."""
    import json

    import torch.multiprocessing as mp

    n, bs = 16, 2  # 8 batches
    mp.spawn(_dynamic_worker, args=(2, _free_port(), n, bs, str(tmp_path), "", ("blocked",), 1), nprocs=2, join=True)
    runs = [json.load(open(tmp_path / f"y{r}.json")) for r in range(2)]
    assert all(z["same"] for z in runs)
    assert len(runs[0]["decoded"]) == 1 and len(runs[1]["decoded"]) == 7, runs


def test_dynamic_schedule_resume_gloo_world2(tmp_path):
    """Dynamic resume: one file per global batch (with the rank that decoded it); after two files are lost the rerun
    decodes exactly those two batches (whichever rank claims them) and returns the same predictions."""
    import json

    import torch.multiprocessing as mp

    n, bs = 13, 2
    ck = str(tmp_path / "ck")
    mp.spawn(_dynamic_worker, args=(2, _free_port(), n, bs, str(tmp_path), ck, (), 1), nprocs=2, join=True)
    files = sorted(f for f in os.listdir(ck) if f.endswith(".npz"))
    assert files == [f"batch_{j:06d}.npz" for j in range(8)]
    first = [json.load(open(tmp_path / f"y{r}.json")) for r in range(2)]
    for j in range(8):
        with np.load(os.path.join(ck, files[j])) as z:
            assert int(z["rank"]) == first[0]["schedule"][j]
    os.remove(os.path.join(ck, files[2]))
    os.remove(os.path.join(ck, files[7]))
    mp.spawn(_dynamic_worker, args=(2, _free_port(), n, bs, str(tmp_path), ck, (), 1), nprocs=2, join=True)
    runs = [json.load(open(tmp_path / f"y{r}.json")) for r in range(2)]
    assert all(z["same"] for z in runs)
    plans = [shard_batches(n, bs, 2, r) for r in range(2)]
    redone = sorted(tuple(b) for z in runs for b in z["decoded"])
    assert redone == sorted([tuple(plans[0][1]), tuple(plans[1][3])])  # global batches 2 and 7
    assert [x for x in runs[0]["schedule"] if x >= 0] and runs[0]["schedule"].count(-1) == 6


@pytest.mark.parametrize("lanes", [1, 2, 3])
def test_dynamic_schedule_single_process(lanes):
    """Without a process group the claims come from a local counter shared by the lanes: same predictions as the
    static plan, every batch once; on_step sees every global batch once, one call at a time."""
    import threading

    ref = pseudo_label(_StubModel(), _features, 23, batch_size=4, pad_token_id=PAD, gather="end")
    m = _LaneStub()
    seen, busy, clash = [], threading.Lock(), []

    def on_step(j, total):
        if not busy.acquire(blocking=False):
            clash.append(j)
            return
        try:
            seen.append((j, total))
        finally:
            busy.release()

    got = pseudo_label(m, _features, 23, batch_size=4, pad_token_id=PAD, gather="end", schedule="dynamic",
                       lanes=lanes, on_step=on_step)
    _same(got, ref)
    assert sorted(seen) == [(j, 6) for j in range(6)] and not clash
    assert sorted(tuple(b) for h in m.lanes for b in h.batches) == sorted(tuple(b) for b in shard_batches(23, 4, 1, 0))
    with pytest.raises(ValueError, match="schedule"):
        pseudo_label(_StubModel(), _features, 3, batch_size=4, pad_token_id=PAD, schedule="dynamic")


def _bench_configs():
    import importlib.util

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_configs", os.path.join(root, "tools", "bench_configs.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_dp_projection_pass_units():
    """VERDICT r5 item 5's seek-pass work units (tools/bench_configs.py pass_unit_makespan): with every batch one
    pass they are the dynamic batch schedule; with multi-pass batches they never lose to it, and on round 4's measured
    config-4 per-batch times (four three-pass batches, the LAST batch among them) W = 8 stays at the dynamic
    schedule's 0.84 -- the last batch's three dependent passes are the job's critical path."""
    bc = _bench_configs()
    rng = np.random.default_rng(3)
    one = 0.4 + 0.01 * rng.random(56)
    p1 = bc.dp_projection(one, passes=[1] * 56)
    for w in ("w2", "w4", "w8"):
        assert p1[w]["dynamic_pass_units"] == p1[w]["dynamic"]
    t = np.full(56, 0.429)
    passes = [1] * 56
    for j in (0, 16, 50, 55):
        t[j], passes[j] = 0.825, 3
    pj = bc.dp_projection(t, passes=passes)
    for w in ("w2", "w4", "w8"):
        assert pj[w]["dynamic_pass_units"] >= pj[w]["dynamic"] - 1e-4
    assert pj["w8"]["dynamic_pass_units"] < 0.86
    # the same batches with the three-pass ones first: the passes then overlap other ranks' work
    order = [0, 16, 50, 55] + [j for j in range(56) if j not in (0, 16, 50, 55)]
    pf = bc.dp_projection(t[order], passes=[passes[j] for j in order])
    assert pf["w8"]["dynamic_pass_units"] > 0.93

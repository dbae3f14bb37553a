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

from kwhisper.pseudo_label import gather_remainder, pseudo_label, shard_batches, write_transcription_csv

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

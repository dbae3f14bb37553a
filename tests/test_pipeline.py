"""ASR pipeline path (kwhisper.pipeline) against transformers' own functions, CPU only.

* ``chunk_iter`` == TF/pipelines/automatic_speech_recognition.py ``chunk_iter`` (windows, strides, is_last);
* ``find_longest_common_sequence`` == tokenization_whisper ``_find_longest_common_sequence`` on
  overlapping random windows;
* ``decode_asr`` == tokenization_whisper ``_decode_asr`` driven by a stub tokenizer (no vocab files
  offline: the stub decodes ids to "[id]" strings and knows the Whisper special ids), over synthetic
  chunk outputs with timestamps, strides, language tokens and prompts.
The GPU end-to-end test lives in test_gpu_generate.py.
"""
import os

import numpy as np
import pytest

from kwhisper.config import LANGUAGES, TINY, generation_constants
from kwhisper.pipeline import chunk_iter, decode_asr, find_longest_common_sequence

asr = pytest.importorskip("transformers.pipelines.automatic_speech_recognition")
tw = pytest.importorskip("transformers.models.whisper.tokenization_whisper")

G = generation_constants(TINY)
TS = G.no_timestamps_token_id + 1


class StubTokenizer:
    """What _decode_asr asks of a Whisper tokenizer, for the multilingual v1/v2 vocabulary."""

    def __init__(self, g=G):
        self.g = g
        self.all_special_ids = list(range(g.eos_token_id, g.no_timestamps_token_id + 1))
        self._names = {g.eos_token_id: "endoftext", g.decoder_start_token_id: "startoftranscript",
                       g.prev_sot_token_id: "startofprev", g.no_timestamps_token_id: "notimestamps",
                       g.task_to_id["translate"]: "translate", g.task_to_id["transcribe"]: "transcribe"}
        for tok, tid in g.lang_to_id.items():
            self._names[tid] = tok[2:-2]

    def convert_tokens_to_ids(self, tok):
        inv = {f"<|{v}|>": k for k, v in self._names.items()}
        return inv[tok]

    def decode(self, ids):
        ids = [int(i) for i in ids]
        if len(ids) == 1 and ids[0] in self._names:
            return f"<|{self._names[ids[0]]}|>"
        return "".join(f"[{i}]" for i in ids)

    def _strip_prompt(self, token_ids, prompt_token_id, decoder_start_token_id):
        return tw.WhisperTokenizer._strip_prompt(self, token_ids, prompt_token_id, decoder_start_token_id)

    @staticmethod
    def _convert_to_list(token_ids):
        return tw.WhisperTokenizer._convert_to_list(token_ids)


def _vocab(tk):
    lang_of = {tid: dict(LANGUAGES)[tok[2:-2]] for tok, tid in G.lang_to_id.items()}
    return dict(timestamp_begin=TS, special_ids=tk.all_special_ids, lang_of=lang_of,
                prompt_token_id=G.prev_sot_token_id, decoder_start_token_id=G.decoder_start_token_id,
                decode=tk.decode)


class _FE:
    sampling_rate = 16000

    def __call__(self, chunk, **kw):
        return {"n": chunk.shape[0]}


@pytest.mark.parametrize("n", [0, 1, 1000, 16000 * 5, 16000 * 15, 16000 * 15 + 1, 16000 * 31, 16000 * 62 + 7])
@pytest.mark.parametrize("cl,sl,sr", [(240000, 40000, 40000), (480000, 80000, 80000), (16000, 4000, 2000),
                                      (100, 0, 0), (100, 50, 50)])
def test_chunk_iter_matches_transformers(n, cl, sl, sr):
    audio = np.zeros(n, dtype=np.float32)
    if cl - sl - sr <= 0:
        return  # the reference raises ("Chunk length must be superior to stride length") before iterating
    want = [(d["is_last"], d["stride"], d["n"]) for d in asr.chunk_iter(audio, _FE(), cl, sl, sr)]
    got = [(last, st, b - a) for a, b, last, st in chunk_iter(n, cl, sl, sr)]
    assert got == want


def _windows(rng, n_total, n_win, overlap, noise):
    seq = rng.integers(0, 500, n_total).tolist()
    step = max(1, n_total // n_win)
    out = []
    for s in range(0, n_total, step):
        w = seq[max(0, s - overlap): s + step + overlap]
        w = [t if rng.random() > noise else int(rng.integers(0, 500)) for t in w]
        out.append(w)
    return out


@pytest.mark.parametrize("seed", range(40))
def test_longest_common_sequence_matches_transformers(seed):
    rng = np.random.default_rng(seed)
    wins = _windows(rng, int(rng.integers(1, 120)), int(rng.integers(1, 6)), int(rng.integers(0, 12)),
                    float(rng.choice([0.0, 0.1, 0.4])))
    if seed % 7 == 0:
        wins.append([])
    assert find_longest_common_sequence(wins) == tw._find_longest_common_sequence(wins)


def _chunk_tokens(rng, with_ts, prompt, lang_tok, L=30):
    toks = []
    if prompt:
        toks += [G.prev_sot_token_id, 11, 12, G.decoder_start_token_id]
    if lang_tok:
        toks += [lang_tok, G.task_to_id["transcribe"]]
    t = 0
    while len(toks) < L:
        if with_ts:
            t += int(rng.integers(0, 60))
            toks.append(TS + min(t, 1500))
            toks += rng.integers(0, 400, int(rng.integers(1, 6))).tolist()
            t += int(rng.integers(0, 80))
            toks.append(TS + min(t, 1500))
            if rng.random() < 0.2 and toks[-1] > TS:
                toks.append(toks[-1])  # duplicate-timestamp quirk
        else:
            toks += rng.integers(0, 400, 4).tolist()
    if rng.random() < 0.3:
        toks.append(G.eos_token_id)
    return np.asarray([toks], dtype=np.int64)


@pytest.mark.parametrize("seed", range(60))
def test_decode_asr_matches_transformers(seed):
    rng = np.random.default_rng(seed)
    tk = StubTokenizer()
    with_ts = bool(seed % 2)
    n_chunks = int(rng.integers(1, 5))
    langs = [G.lang_to_id["<|ja|>"], G.lang_to_id["<|en|>"], None]
    outputs = []
    for c in range(n_chunks):
        lt = langs[int(rng.integers(0, 3))] if seed % 3 == 0 else None
        o = {"tokens": _chunk_tokens(rng, with_ts, prompt=(seed % 5 == 0 and c == 0), lang_tok=lt)}
        if seed % 4 != 1:  # strided (chunked) or not
            left = 0.0 if c == 0 else 2.5
            right = 0.0 if c == n_chunks - 1 else 2.5
            o["stride"] = (15.0, left, right)
        outputs.append(o)
    rl = seed % 3 == 0
    ref_outputs = [dict(o) for o in outputs]
    want = tw._decode_asr(tk, ref_outputs, return_timestamps=with_ts, return_language=rl, time_precision=0.02)
    got = decode_asr([dict(o) for o in outputs], return_timestamps=with_ts, return_language=rl,
                     time_precision=0.02, **_vocab(tk))
    assert got == want


def test_decode_asr_token_mode():
    """Without a tokenizer the merge returns token ids (the text of each chunk is its id list)."""
    tk = StubTokenizer()
    rng = np.random.default_rng(3)
    outputs = [{"tokens": _chunk_tokens(rng, False, False, None), "stride": (15.0, 0.0 if c == 0 else 2.5,
                                                                             2.5 if c < 2 else 0.0)}
               for c in range(3)]
    v = _vocab(tk)
    text, _ = decode_asr(outputs, return_timestamps=False, time_precision=0.02, **v)
    v["decode"] = None
    toks, _ = decode_asr(outputs, return_timestamps=False, time_precision=0.02, **v)
    assert text == tk.decode(toks)


def test_pipeline_generation_defaults_match_transformers():
    """ASRPipeline decodes with the generation config transformers' pipeline builds (base.py:886-907 over
    automatic_speech_recognition.py:160-163): beam 5 by default, max_new_tokens dropped for Whisper's
    max_length 448 and kept (256) when the model leaves max_length at the global default."""
    import torch
    from transformers import GenerationConfig, WhisperConfig, WhisperFeatureExtractor, WhisperForConditionalGeneration
    from transformers import pipeline as hf_pipeline

    from kwhisper.pipeline import ASRPipeline

    cfg = WhisperConfig(vocab_size=51865, d_model=64, encoder_layers=1, decoder_layers=1, encoder_attention_heads=1,
                        decoder_attention_heads=1, encoder_ffn_dim=64, decoder_ffn_dim=64)
    m = WhisperForConditionalGeneration(cfg).eval()
    for max_length in (448, None):
        d = {k: v for k, v in G.to_dict().items() if k not in ("language", "task")}
        d["max_length"] = max_length
        if max_length is None:
            d.pop("max_length")
        m.generation_config = GenerationConfig(**d)

        class _Tok(StubTokenizer):
            pad_token_id, eos_token_id, padding_side = G.pad_token_id, G.eos_token_id, "right"

        p = hf_pipeline("automatic-speech-recognition", model=m, tokenizer=_Tok(), feature_extractor=WhisperFeatureExtractor(),
                        device="cpu")
        ours = G.copy()
        ours.max_length = max_length
        got = ASRPipeline._pipeline_generation_config(ours)
        assert got.num_beams == p.generation_config.num_beams == 5
        assert got.pipeline_max_new_tokens == p.generation_config.max_new_tokens, max_length


# ---- data-parallel pipeline (config 5 at W GPUs) -----------------------------------------
class _StubFE:
    """Feature-extractor stand-in (CPU): one 2-value 'frame' per window -- its sample count and a checksum."""

    sampling_rate, n_samples, padding_value, chunk_length, hop_length = 16000, 480000, 0.0, 30, 160
    device = "cpu"

    def __call__(self, audios, sampling_rate=None, return_attention_mask=None, **kw):
        import torch

        f = torch.tensor([[[len(a), float(np.round(np.abs(a).sum() * 1e3))]] for a in audios], dtype=torch.float32)
        return {"input_features": f, "attention_mask": torch.ones((len(audios), 1), dtype=torch.int32)}


class _StubASRModel:
    """generate(): a deterministic token row per window (1-4 tokens), right-padded to the batch's longest."""

    class config:  # noqa: N801
        max_source_positions, num_mel_bins = 1500, 80

    device = "cpu"

    def __init__(self):
        self.generation_config = G.copy()
        self.calls = 0

    def generate(self, feats, attention_mask=None, **kw):
        import torch

        self.calls += 1
        keys = [int(f[0, 0]) * 7 + int(f[0, 1]) for f in feats]
        rows = [[100 + (k % 50) + j for j in range(1 + k % 4)] for k in keys]
        T = max(len(r) for r in rows)
        out = torch.full((len(rows), T), G.pad_token_id, dtype=torch.int64)
        for i, r in enumerate(rows):
            out[i, : len(r)] = torch.tensor(r)
        return out


_DP_CLIPS = [7.0, 40.0, 22.0, 15.0, 31.0, 3.5]


def _dp_clips():
    rng = np.random.default_rng(5)
    return [{"array": (rng.random(int(s * 16000)) - 0.5).astype(np.float32), "sampling_rate": 16000} for s in _DP_CLIPS]


def _dp_pipe_worker(rank, world, port, out_dir):
    import json

    import torch.distributed as dist

    from kwhisper.pipeline import ASRPipeline

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        m = _StubASRModel()
        got = ASRPipeline(m, feature_extractor=_StubFE(), chunk_length_s=15, batch_size=2,
                          data_parallel=True)(_dp_clips())
        with open(os.path.join(out_dir, f"p{rank}.json"), "w") as f:
            json.dump({"res": got, "calls": m.calls}, f, default=lambda x: x.tolist() if hasattr(x, "tolist") else x)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_pipeline_data_parallel_gloo_matches_single_process(tmp_path, world):
    """ASRPipeline under a process group: window batch j runs on rank j % W, one gather at the end, every rank's
    merged output equals the single-process run's, and each rank decoded only its share of the batches."""
    import json
    import socket

    import torch.multiprocessing as mp

    from kwhisper.pipeline import ASRPipeline

    m1 = _StubASRModel()
    want = json.loads(json.dumps(ASRPipeline(m1, feature_extractor=_StubFE(), chunk_length_s=15, batch_size=2)(_dp_clips()),
                                 default=lambda x: x.tolist() if hasattr(x, "tolist") else x))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_dp_pipe_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    calls = []
    for r in range(world):
        z = json.load(open(tmp_path / f"p{r}.json"))
        assert z["res"] == want
        calls.append(z["calls"])
    assert sum(calls) == m1.calls and max(calls) - min(calls) <= 1


def _dp_mismatch_worker(rank, world, port, out_dir, mode="reversed"):
    import torch.distributed as dist

    from kwhisper.pipeline import ASRPipeline

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        clips = _dp_clips()
        if rank == 1 and mode == "reversed":  # a per-rank shard of the inputs: another clip in position 2 (same window count)
            clips[2] = {"array": clips[2]["array"][::-1].copy(), "sampling_rate": 16000}
        elif rank == 1:  # the same edges (silent start and end), different audio in the middle of a window
            for c in clips:
                c["array"][:4000] = 0.0
                c["array"][-4000:] = 0.0
            a = clips[1]["array"].copy()
            a[len(a) // 2] += 0.25
            clips[1] = {"array": a, "sampling_rate": 16000}
        if mode == "middle" and rank == 0:
            for c in clips:
                c["array"][:4000] = 0.0
                c["array"][-4000:] = 0.0
        msg, m = "", _StubASRModel()
        try:
            ASRPipeline(m, feature_extractor=_StubFE(), chunk_length_s=15, batch_size=2, data_parallel=True)(clips)
        except ValueError as e:
            msg = str(e)
        # data_parallel off (the default): each rank decodes its own inputs, no collective
        ASRPipeline(m, feature_extractor=_StubFE(), chunk_length_s=15, batch_size=2)(clips)
        with open(os.path.join(out_dir, f"m{rank}.txt"), "w") as f:
            f.write(msg)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["reversed", "middle"])
def test_pipeline_data_parallel_refuses_different_inputs(tmp_path, mode):
    """data_parallel is opt-in, and with it every rank must pass the same inputs -- ranks holding
    different audio raise ValueError on every rank (before any window batch is split or gathered).  ADVICE r05
    ("middle"): the ranks' clips share silent starts and ends and differ in one sample in the middle of a window,
    which a digest of the window edges alone would miss."""
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_dp_mismatch_worker, args=(2, port, str(tmp_path), mode), nprocs=2, join=True)
    for r in range(2):
        assert "same inputs on every rank" in open(tmp_path / f"m{r}.txt").read()


class _LaneASRModel(_StubASRModel):
    """A stub with lane(): every handle counts its own generate() calls."""

    def __init__(self, handles=None):
        super().__init__()
        self.handles = handles if handles is not None else [self]

    def lane(self):
        other = _LaneASRModel(self.handles)
        self.handles.append(other)
        return other


@pytest.mark.parametrize("lanes", [2, 3])
def test_pipeline_lanes_match_one_lane(lanes):
    """ASRPipeline(lanes=n): window batches decode on n model handles from n host threads; the merged output equals
    the one-lane run's, every batch is decoded exactly once, and a second call reuses the same handles."""
    import json

    from kwhisper.pipeline import ASRPipeline

    enc = lambda r: json.loads(json.dumps(r, default=lambda x: x.tolist() if hasattr(x, "tolist") else x))  # noqa: E731
    m1 = _StubASRModel()
    want = enc(ASRPipeline(m1, feature_extractor=_StubFE(), chunk_length_s=15, batch_size=2)(_dp_clips()))
    m = _LaneASRModel()
    pipe = ASRPipeline(m, feature_extractor=_StubFE(), chunk_length_s=15, batch_size=2, lanes=lanes)
    for _ in range(2):
        assert enc(pipe(_dp_clips())) == want
    assert len(m.handles) == lanes
    assert sum(h.calls for h in m.handles) == 2 * m1.calls
    with pytest.raises(ValueError, match="lane"):
        ASRPipeline(_StubASRModel(), feature_extractor=_StubFE(), lanes=2)


def _dp_lanes_worker(rank, world, port, out_dir):
    import json

    import torch.distributed as dist

    from kwhisper.pipeline import ASRPipeline

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        m = _LaneASRModel()
        got = ASRPipeline(m, feature_extractor=_StubFE(), chunk_length_s=15, batch_size=1, lanes=2,
                          data_parallel=True)(_dp_clips())
        with open(os.path.join(out_dir, f"l{rank}.json"), "w") as f:
            json.dump({"res": got, "calls": sum(h.calls for h in m.handles)}, f,
                      default=lambda x: x.tolist() if hasattr(x, "tolist") else x)
    finally:
        dist.destroy_process_group()


def test_pipeline_data_parallel_with_lanes_gloo():
    """Both at once: window batches round-robin over two gloo ranks, each rank decoding its share on two lanes;
    every rank's merged output equals the single-process, single-lane run's."""
    import json
    import socket
    import tempfile

    import torch.multiprocessing as mp

    from kwhisper.pipeline import ASRPipeline

    m1 = _StubASRModel()
    want = json.loads(json.dumps(ASRPipeline(m1, feature_extractor=_StubFE(), chunk_length_s=15, batch_size=1)(_dp_clips()),
                                 default=lambda x: x.tolist() if hasattr(x, "tolist") else x))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_dp_lanes_worker, args=(2, port, d), nprocs=2, join=True)
        calls = 0
        for r in range(2):
            z = json.load(open(os.path.join(d, f"l{r}.json")))
            assert z["res"] == want
            calls += z["calls"]
    assert calls == m1.calls

#!/usr/bin/env python
"""Lab A/B (not product): the decode step's tail -- LM head + greedy sampler (+ embed) -- as kw_dec_lm_greedy (one
launch) vs kw_dec_linear + kw_greedy_step, on the bench workload (large-v3, B = 32, 128 tokens, bench.py's weights).
Alternates the two in rounds on one box: per round the step graph's replay time (HIP events, 200 replays) and one
whole generate() batch.  Tokens must be identical.

    python tools/lab/tail_ab.py [--rounds 3]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kotoba-whisper_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--replays", type=int, default=124)
    a = ap.parse_args()
    from kwhisper.config import LARGE_V3
    from kwhisper.feature_extraction import WhisperFeatureExtractor
    from kwhisper.generation import KWhisperForConditionalGeneration
    from kwhisper.synthetic import dummy_audio, synthetic_state_dict_torch

    dev = torch.device("cuda", 0)
    sd = synthetic_state_dict_torch(LARGE_V3, seed=0, device=dev)
    model = KWhisperForConditionalGeneration.from_state_dict(LARGE_V3, sd, dtype=torch.bfloat16, device=dev)
    del sd
    fe = WhisperFeatureExtractor(feature_size=LARGE_V3.num_mel_bins, device=dev)
    B = 32
    audio = torch.from_numpy(np.stack([dummy_audio(i) for i in range(B)])).to(dev)
    kw = dict(language="ja", task="transcribe", max_length=128, return_timestamps=False)
    feats = fe.extract(audio)
    eng = model.engine
    toks, res = {}, {True: [], False: []}
    for r in range(a.rounds):
        for fuse in (False, True):
            eng.fuse_lm_greedy = fuse
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = model.generate(feats, **kw)
            torch.cuda.synchronize()
            t_gen = time.perf_counter() - t0
            sess = model._sessions[(B, 1)]
            assert sess.lm_greedy_last == fuse
            toks.setdefault(fuse, out.cpu())
            g = sess._graph
            sess.cur_len.fill_(4)  # replays advance the device position: 4 .. 4 + replays (< 256, qkv_self's range)
            s = torch.cuda.current_stream()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            g.replay()
            e0.record(s)
            for _ in range(a.replays - 1):
                g.replay()
            e1.record(s)
            e1.synchronize()
            step_us = e0.elapsed_time(e1) / a.replays * 1e3
            res[fuse].append({"step_us": round(step_us, 2), "generate_ms": round(t_gen * 1e3, 2)})
            print(f"round {r} fuse={fuse}: step {step_us:.2f} us, generate {t_gen * 1e3:.1f} ms", flush=True)
    same = torch.equal(toks[True], toks[False])
    print(json.dumps({"tokens_identical": same, "fused": res[True], "two_launch": res[False]}))
    assert same


if __name__ == "__main__":
    main()

#!/usr/bin/env python
"""Record the engine's own seek-loop trajectory on a fixture's features (GPU box), for a teacher-forced fixture.

On the HIP log-mel of config-4 stand-in clips 1 and 522 (tests/golden/large_v3_c4_hipmel.npz), transformers' fp32
and bf16 large-v3 decode every row in ONE seek pass, while the bf16 engine -- whose greedy choices follow fp32's only
where fp32 decides by a margin above the bf16 noise -- takes three on some rows (profiles/r04t_config4.json).  This
runs generate() with the config-4 settings (run_pseudo_labelling.py:99-102,338) in the given dtypes and writes every
pass: the rows, their seek and frame count, and the decoded ids with the prompt.  tools/make_fixtures.py --only
c4_traj then has transformers fp32 score exactly those passes (teacher-forced), so a GPU test can hold the engine's
own passes 2 and 3 to fp32's choices wherever fp32 is confident.

    python tools/dump_trajectory.py --fixture tests/golden/large_v3_c4_hipmel.npz --out gpurun_out/c4_traj.npz
"""
from __future__ import annotations

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kotoba-whisper_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fixture", default="tests/golden/large_v3_c4_hipmel.npz")
    ap.add_argument("--dtypes", default="bfloat16,float32")
    ap.add_argument("--out", default="gpurun_out/c4_traj.npz")
    a = ap.parse_args()
    from kwhisper.config import LARGE_V3, generation_constants
    from kwhisper.generation import KWhisperForConditionalGeneration
    from kwhisper.synthetic import synthetic_state_dict

    g = np.load(a.fixture)
    feats = torch.from_numpy(g["features"]).cuda()
    kw = dict(language="ja", task="transcribe", return_timestamps=True, max_length=int(g["max_length"]))
    out = {}
    for name in a.dtypes.split(","):
        m = KWhisperForConditionalGeneration.from_state_dict(
            LARGE_V3, synthetic_state_dict(LARGE_V3, 0), dtype=getattr(torch, name),
            generation_config=generation_constants(LARGE_V3))
        m.record_pass_ids = True
        toks = m.generate(feats, **kw).cpu().numpy()
        st = m.stats
        rows, seeks, nfr, it, seqs = [], [], [], [], []
        for k, ((r, s, n), ids) in enumerate(zip(st["pass_log"], st["pass_ids"])):
            rows += r
            seeks += s
            nfr += n
            it += [k] * len(r)
            seqs += list(ids)
        T = max(len(x) for x in seqs)
        seq = np.full((len(seqs), T), -1, np.int64)
        for i, x in enumerate(seqs):
            seq[i, : len(x)] = x
        tag = {"bfloat16": "bf16", "float32": "fp32"}[name]
        out.update({f"{tag}_tokens": toks, f"{tag}_passes": st["row_passes"], f"{tag}_pass_iter": np.array(it),
                    f"{tag}_pass_row": np.array(rows), f"{tag}_pass_seek": np.array(seeks),
                    f"{tag}_pass_nframes": np.array(nfr), f"{tag}_pass_seq": seq})
        print(f"{name}: passes per row {st['row_passes'].tolist()}", flush=True)
        del m
        torch.cuda.empty_cache()
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    np.savez_compressed(a.out, **out)
    print(f"wrote {a.out}", flush=True)


if __name__ == "__main__":
    main()

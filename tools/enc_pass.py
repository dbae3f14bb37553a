#!/usr/bin/env python
"""The large-v3 B = 32 encoder as the bench runs it, for counter passes (development tool): ``--streams 1`` runs the
one-pass encoder (every GEMM / attention launch alone on the chip, so per-kernel counters are clean), ``--streams 2``
the bench's two-row-block overlap.  Prints ms per pass.

    rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/x -o run \\
        -- python3 tools/enc_pass.py --streams 1
"""
from __future__ import annotations

import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kotoba-whisper_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=1)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    from kwhisper.config import PRESETS
    from kwhisper.engine import WhisperEngine
    from kwhisper.synthetic import synthetic_state_dict_torch

    dev = torch.device("cuda")
    shape = PRESETS["large-v3"]
    sd = synthetic_state_dict_torch(shape, seed=0, device=dev)
    eng = WhisperEngine(shape, sd, dtype=torch.bfloat16, device=dev, encoder_streams=a.streams)
    del sd
    torch.cuda.empty_cache()
    mel = torch.randn(32, shape.num_mel_bins, shape.n_frames, device=dev) * 0.5
    eng.encode(mel)
    torch.cuda.synchronize()
    for _ in range(a.reps):
        t0 = time.perf_counter()
        eng.encode(mel)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        print(f"encoder pass ({a.streams} stream(s)): {ms:.2f} ms = {2.2738e12 * 32 / ms / 1e9:.0f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()

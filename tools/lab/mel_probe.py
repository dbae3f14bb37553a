#!/usr/bin/env python
"""kw_log_mel time at the bench's shape (large-v3: 128 mels, B = 32 clips of 30 s), 20 launches (lab r05ac)."""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kotoba-whisper_amd"))

import torch  # noqa: E402

from kwhisper.config import LARGE_V3  # noqa: E402
from kwhisper.feature_extraction import WhisperFeatureExtractor  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    fe = WhisperFeatureExtractor(feature_size=LARGE_V3.num_mel_bins, device=dev)
    audio = (torch.rand(32, 480000, device=dev) - 0.5) * 0.014
    out = fe.extract(audio)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        out = fe.extract(audio)
    e1.record()
    e1.synchronize()
    print(json.dumps({"log_mel_ms": round(e0.elapsed_time(e1) / 20, 3), "checksum": float(out.double().sum())}))


if __name__ == "__main__":
    main()

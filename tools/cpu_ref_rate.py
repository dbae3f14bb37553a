#!/usr/bin/env python
"""The reference's CPU path at a full batch, for anchoring bench.py's bounded cpu_baseline sample:
transformers 5.15.0 WhisperForConditionalGeneration.generate, fp32, on the host cores
(oracle/cpu_baseline.py; run_speed_eval.py:73-78 timing).  One JSON line.
    python tools/cpu_ref_rate.py --batch 32 [--threads N] [--model large-v3] [--max-length 128]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "kotoba-whisper_amd"))

from kwhisper.config import PRESETS  # noqa: E402
from oracle.cpu_baseline import hf_cpu_generate_rate  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=32)
ap.add_argument("--threads", type=int, default=None)
ap.add_argument("--model", default="large-v3")
ap.add_argument("--max-length", type=int, default=128)
a = ap.parse_args()
r = hf_cpu_generate_rate(PRESETS[a.model], a.batch, a.max_length, threads=a.threads)
r.update(model=a.model, omp_num_threads=os.environ.get("OMP_NUM_THREADS"),
         workload="config 3 on CPU: greedy, language ja, transcribe, no timestamps, 30 s noise clips")
print(json.dumps(r), flush=True)

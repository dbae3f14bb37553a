#!/usr/bin/env python
"""Batch-1 pipeline latency in the schema of the reference's run_speed_eval.py (development tool).

Restates /root/reference/run_speed_eval.py:14-88 on the MI355X engine: a `duration`-second noise clip
((rand - 0.5) * 2 * 0.007, :14-17) through the ASR pipeline with chunk_length_s=15 (:56-59) and batch size 1,
n_trial + 1 calls with the first dropped (:73-77), printed as one runtime_pipeline.jsonl line (:78).
The reference publishes whisper-large-v3 30 s at 0.182 s (eval_pipeline/runtime_pipeline.jsonl:79, bf16 sdpa
on an NVIDIA GPU, real weights).  Random weights never emit EOS, so the decode here is bounded by
``--max-new-tokens`` per window (stated in the line): a real checkpoint stops after a few tokens on noise.

    python tools/speed_eval.py --model large-v3 --duration 30 --max-new-tokens 16 >> profiles/<tag>_runtime_pipeline.jsonl
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from statistics import mean, stdev
from time import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kotoba-whisper_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="large-v3")
    ap.add_argument("--language", default="en")
    ap.add_argument("--task", default="transcribe")
    ap.add_argument("-n", "--n-trial", type=int, default=15)
    ap.add_argument("-d", "--duration", type=int, default=30)
    ap.add_argument("--max-new-tokens", type=int, default=16)
    ap.add_argument("--num-beams", type=int, default=5, help="the pipeline's default (TF/pipelines/"
                                                             "automatic_speech_recognition.py:160-163)")
    a = ap.parse_args()
    from kwhisper.config import PRESETS
    from kwhisper.generation import KWhisperForConditionalGeneration
    from kwhisper.pipeline import ASRPipeline
    from kwhisper.synthetic import synthetic_state_dict_torch

    dev = torch.device("cuda")
    shape = PRESETS[a.model]
    sd = synthetic_state_dict_torch(shape, seed=0, device=dev)
    model = KWhisperForConditionalGeneration.from_state_dict(shape, sd, dtype=torch.bfloat16, device=dev)
    del sd
    pipe = ASRPipeline(model, chunk_length_s=15, batch_size=1,
                       generate_kwargs=dict(language=a.language, task=a.task, num_beams=a.num_beams,
                                            max_new_tokens=a.max_new_tokens))
    rng = np.random.default_rng(0)
    audio = {"array": ((rng.random(a.duration * 16000) - 0.5) * 2 * 0.007).astype(np.float32), "sampling_rate": 16000}
    elapsed = []
    for _ in range(a.n_trial + 1):
        torch.cuda.synchronize()
        start = time()
        pipe(dict(audio))
        torch.cuda.synchronize()
        elapsed.append(time() - start)
    elapsed = elapsed[1:]
    print(json.dumps({
        "model": f"openai/whisper-{a.model} (random-init weights, kwhisper bf16 on MI355X)", "attention": "kwhisper",
        "device": "cuda:0", "duration": a.duration, "time (mean)": mean(elapsed), "time (std)": stdev(elapsed),
        "time (all)": elapsed, "chunk_length_s": 15, "batch_size": 1, "num_beams": a.num_beams,
        "max_new_tokens_per_window": a.max_new_tokens, "language": a.language, "task": a.task,
        "reference": "run_speed_eval.py:14-88; published large-v3 30 s: 0.182 s (runtime_pipeline.jsonl:79)"}))


if __name__ == "__main__":
    main()

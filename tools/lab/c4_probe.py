#!/usr/bin/env python
"""Lab: which audio for the config-4 fixture exercises the timestamp path best?  The fp32 engine is bit-exact
with HF fp32 (tests), so it previews on the GPU what tools/make_fixtures.py would record on the CPU: distinct
rows, timestamp tokens per row and seek passes for the ReazonSpeech-length stand-in clips with different
content (noise as run_speed_eval.py, the louder tone clips cut to the same durations)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "kotoba-whisper_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from kwhisper import synthetic as S  # noqa: E402
from kwhisper.config import LARGE_V3, generation_constants  # noqa: E402
from kwhisper.generation import KWhisperForConditionalGeneration  # noqa: E402
from oracle.mel import log_mel, pad_or_trim  # noqa: E402


def variants(n=32):
    d = S.reazon_durations()[:n]
    out = {"noise": [S.reazon_audio(i, float(x)) for i, x in enumerate(d)],
           "tone": [S.tone_audio(i)[: int(float(x) * 16000)] for i, x in enumerate(d)],
           "tone_x8": [S.tone_audio(i % 8)[: int(float(x) * 16000)] * 0.5 for i, x in enumerate(d)]}
    mix = []
    for i, x in enumerate(d):
        mix.append(out["tone"][i] if i % 2 else out["noise"][i])
    out["mix"] = mix
    return out


def main():
    t0 = time.time()
    dtype = torch.float32 if "--bf16" not in sys.argv else torch.bfloat16
    m = KWhisperForConditionalGeneration.from_state_dict(LARGE_V3, S.synthetic_state_dict(LARGE_V3, 0), dtype=dtype,
                                                         generation_config=generation_constants(LARGE_V3))
    print(f"model {time.time() - t0:.1f}s", flush=True)
    gold = os.path.join(ROOT, "tests", "golden", "large_v3_ts_b32_fp32.npz")
    for name, audio in variants().items():
        feats = torch.from_numpy(log_mel(np.stack([pad_or_trim(a) for a in audio]), 128)).cuda()
        t1 = time.time()
        toks = m.generate(feats, language="ja", task="transcribe", return_timestamps=True, max_length=128)
        toks = toks.cpu().numpy()
        res = {"variant": name, "seconds": round(time.time() - t1, 2), "passes": m.stats.get("passes"),
               "shape": list(toks.shape), "distinct_rows": len({tuple(r) for r in toks}),
               "ts_per_row": (toks >= 50365).sum(1).tolist(),
               "distinct_tokens_per_row": [len(set(r.tolist())) for r in toks]}
        if name == "noise" and os.path.exists(gold) and dtype == torch.float32:
            g = np.load(gold)
            res["equals_hf_fixture"] = bool(toks.shape == g["tokens"].shape and (toks == g["tokens"]).all())
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

"""A/B timing of the encoder attention kernel and the whole encoder (development): run once per library
build, e.g.  KWHISPER_LIB=.../libkw_old.so python tools/lab/attn_ab.py ; also checks the output against a
torch fp32 reference of the same attention."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kotoba-whisper_amd"))
import torch  # noqa: E402

from kwhisper import ops  # noqa: E402
from kwhisper.config import PRESETS  # noqa: E402
from kwhisper.engine import WhisperEngine  # noqa: E402
from kwhisper.synthetic import synthetic_state_dict_torch  # noqa: E402

dev = torch.device("cuda")
B, H, T, hd = 32, 20, 1500, 64
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def tm(fn, n=10):
    fn()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


res = {"lib": os.environ.get("KWHISPER_LIB", "default")}
for scale in (0.5, 2.0):
    qkv = (torch.randn(3, B, H, T, hd, device=dev) * scale).bfloat16()
    qkv[0] *= 0.125
    out = torch.empty(B * T, H * hd, device=dev, dtype=torch.bfloat16)
    res[f"attn_us_scale{scale}"] = round(tm(lambda: ops.attention(qkv, B, H, T, hd, out)), 1)
    q, k, v = (qkv[i, :2].float() for i in range(3))
    ref = torch.softmax(q @ k.transpose(-1, -2), -1) @ v  # (2, H, T, hd)
    got = out.view(B, T, H, hd)[:2].permute(0, 2, 1, 3).float()
    res[f"attn_maxerr_scale{scale}"] = float((got - ref).abs().max())
shape = PRESETS["large-v3"]
sd = synthetic_state_dict_torch(shape, seed=0, device=dev)
eng = WhisperEngine(shape, sd, dtype=torch.bfloat16, device=dev)
del sd
feats = torch.randn(B, shape.num_mel_bins, 3000, device=dev)
res["encoder_ms"] = round(tm(lambda: eng.encode(feats), 3) / 1e3, 2)
print(res, flush=True)

"""r03aq lab: the two-block encoder with unequal blocks (engine._lab_enc_sizes): 16+16, 18+14, 20+12, 24+8 at
large-v3 B = 32; bitwise vs one pass, HIP events, alternating rounds."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kotoba-whisper_amd"))
import torch  # noqa: E402

from kwhisper.config import PRESETS  # noqa: E402
from kwhisper.generation import KWhisperForConditionalGeneration  # noqa: E402
from kwhisper.synthetic import synthetic_state_dict_torch  # noqa: E402

dev = torch.device("cuda")
shape = PRESETS["large-v3"]
sd = synthetic_state_dict_torch(shape, seed=0, device=dev)
eng = KWhisperForConditionalGeneration.from_state_dict(shape, sd, dtype=torch.bfloat16, device=dev).engine
del sd
torch.cuda.empty_cache()
mel = torch.randn(32, shape.num_mel_bins, shape.n_frames, device=dev) * 0.5
eng.encoder_streams = 1
ref = eng.encode(mel).clone()
eng.encoder_streams = 2
cases = [(16, 16), (18, 14), (20, 12), (24, 8)]
for c in cases:
    eng._lab_enc_sizes = c
    print(c, "bitwise", torch.equal(ref.view(torch.int16), eng.encode(mel).view(torch.int16)), flush=True)
best = {}
for _ in range(4):
    for c in cases:
        eng._lab_enc_sizes = c
        eng.encode(mel)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            eng.encode(mel)
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1) / 3
        best[c] = min(best.get(c, 1e9), ms)
        print(f"{c}: {ms:.2f} ms", flush=True)
print({str(k): round(v, 2) for k, v in best.items()})

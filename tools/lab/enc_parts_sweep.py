"""r03ag lab: engine.encode at large-v3 B = 32 with encoder_streams = 1, 2, 3, 4 (batch parts on side streams),
bitwise against the one-pass encoder, HIP events, alternating rounds."""
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
for n in (2, 3, 4):
    eng.encoder_streams = n
    print(f"parts {n}: bitwise", torch.equal(ref.view(torch.int16), eng.encode(mel).view(torch.int16)), flush=True)
best = {}
for _ in range(4):
    for n in (1, 2, 3, 4):
        eng.encoder_streams = n
        eng.encode(mel)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            eng.encode(mel)
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1) / 3
        best[n] = min(best.get(n, 1e9), ms)
        print(f"parts {n}: {ms:.2f} ms", flush=True)
print({k: round(v, 2) for k, v in best.items()})

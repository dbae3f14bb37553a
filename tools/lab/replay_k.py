"""r03al lab: greedy generate() end to end at large-v3 B = 32 (128 new tokens) with 1 vs 2 decode steps per
hipGraph replay (WhisperEngine.steps_per_replay); tokens compared, wall time per batch (alternating rounds)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kotoba-whisper_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from kwhisper.config import PRESETS  # noqa: E402
from kwhisper.feature_extraction import WhisperFeatureExtractor  # noqa: E402
from kwhisper.generation import KWhisperForConditionalGeneration  # noqa: E402
from kwhisper.synthetic import dummy_audio, synthetic_state_dict_torch  # noqa: E402

dev = torch.device("cuda")
shape = PRESETS["large-v3"]
sd = synthetic_state_dict_torch(shape, seed=0, device=dev)
model = KWhisperForConditionalGeneration.from_state_dict(shape, sd, dtype=torch.bfloat16, device=dev)
del sd
torch.cuda.empty_cache()
fe = WhisperFeatureExtractor(feature_size=shape.num_mel_bins, device=dev)
audio = torch.from_numpy(np.stack([dummy_audio(i) for i in range(32)])).to(dev)
kw = dict(language="ja", task="transcribe", max_length=128, return_timestamps=False)
eng = model.engine
KS = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1,2").split(",")]
ids, best = {}, {}
for k in KS:
    eng.steps_per_replay = k
    ids[k] = model.generate(fe.extract(audio), **kw).cpu()
print("tokens equal:", all(torch.equal(ids[KS[0]], ids[k]) for k in KS), flush=True)
for _ in range(4):
    for k in KS:
        eng.steps_per_replay = k
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            model.generate(fe.extract(audio), **kw)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / 3 * 1e3
        best[k] = min(best.get(k, 1e9), ms)
        print(f"steps per replay {k}: {ms:.2f} ms per batch ({32 * 30 / ms * 1e3:.1f} audio-s/s)", flush=True)
print({k: round(v, 2) for k, v in best.items()})

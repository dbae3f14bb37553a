"""r03ah lab: the greedy prefill (4-token prompt, large-v3, B = 32) as one pass vs two row blocks on two side
streams (WhisperEngine.prefill_streams): token ids of generate() bitwise, and the captured prefill graph's replay
time (HIP events, alternating rounds)."""
import os
import sys

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
B = 32
audio = torch.from_numpy(np.stack([dummy_audio(i) for i in range(B)])).to(dev)
feats = fe.extract(audio)
kw = dict(language="ja", task="transcribe", max_length=128, return_timestamps=False)
ids = {}
eng = model.engine
for parts in (1, 2, 1, 2):
    eng.prefill_streams = parts
    ids.setdefault(parts, []).append(model.generate(feats, **kw).cpu())
sess = model._sessions.get((B, 1)) or model._sessions[(B, 1, 1)]
print("ids equal across runs / settings:", all(torch.equal(ids[1][0], x) for x in ids[1] + ids[2]), tuple(ids[1][0].shape),
      flush=True)
best = {}
for _ in range(5):
    for parts in (1, 2):
        eng.prefill_streams = parts
        model.generate(feats, **kw)
        pg = next(c["prefill_graph"] for k, c in sess._greedy_cfg.items() if k[-1] == parts and c.get("prefill_graph"))
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            pg.replay()
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1) / 5
        best[parts] = min(best.get(parts, 1e9), ms)
        print(f"prefill graph, {parts} part(s): {ms:.3f} ms", flush=True)
print({k: round(v, 3) for k, v in best.items()})

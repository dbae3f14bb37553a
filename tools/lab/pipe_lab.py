"""Per-batch wall times of generate_pipelined vs generate (development): where does the overlap go?"""
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
fe = WhisperFeatureExtractor(feature_size=shape.num_mel_bins, device=dev)
audio = torch.from_numpy(np.stack([dummy_audio(i) for i in range(32)])).to(dev)
kw = dict(language="ja", task="transcribe", max_length=128, return_timestamps=False)
cus = int(os.environ.get("CUS", "128"))
for mode in ("seq", "pipe", "seq", "pipe"):
    n = 5
    it = (model.generate(fe.extract(audio), **kw) for _ in range(n)) if mode == "seq" else \
        model.generate_pipelined((audio for _ in range(n)), feature_extractor=fe, encoder_cus=cus, **kw)
    ts = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in it:
        t1 = time.perf_counter()
        ts.append(round((t1 - t0) * 1e3, 1))
        t0 = t1
    print(mode, ts, flush=True)

"""r03al debug: tiny bf16 greedy with 1 / 2 decode steps per replay; per-replay device state."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kotoba-whisper_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

from kwhisper.config import TINY, generation_constants  # noqa: E402
from kwhisper.generation import KWhisperForConditionalGeneration  # noqa: E402
from kwhisper.synthetic import synthetic_state_dict  # noqa: E402
import kwhisper.decode as D  # noqa: E402

m = KWhisperForConditionalGeneration.from_state_dict(TINY, synthetic_state_dict(TINY, 0), dtype=torch.bfloat16,
                                                     generation_config=generation_constants(TINY))
g = torch.Generator(device="cuda").manual_seed(9)
feats = torch.randn(6, TINY.num_mel_bins, TINY.n_frames, device="cuda", generator=g) * 0.5
kw = dict(language="ja", task="transcribe", return_timestamps=False, max_length=25)
orig = torch.cuda.CUDAGraph.replay


def traced(self):
    orig(self)
    torch.cuda.synchronize()
    s = next(iter(m._sessions.values()))
    print("  replay: cur_len", int(s.cur_len.item()), "n_unfinished", int(s.n_unfinished.item()),
          "unfinished", s.unfinished.tolist(), flush=True)


torch.cuda.CUDAGraph.replay = traced
for k in (2, 1):
    m.engine.steps_per_replay = k
    print("K", k, flush=True)
    out = m.generate(feats, **kw)
    print("K", k, "shape", tuple(out.shape), flush=True)

"""Prefill (P = 4 prompt tokens) vs one decode step, large-v3 B = 32 (development)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kotoba-whisper_amd"))
import torch  # noqa: E402

from kwhisper.config import PRESETS  # noqa: E402
from kwhisper.engine import WhisperEngine  # noqa: E402
from kwhisper.synthetic import synthetic_state_dict_torch  # noqa: E402

dev = torch.device("cuda")
shape = PRESETS["large-v3"]
sd = synthetic_state_dict_torch(shape, seed=0, device=dev)
eng = WhisperEngine(shape, sd, dtype=torch.bfloat16, device=dev)
del sd
B = int(os.environ.get("B", "32"))
T, d = shape.max_source_positions, shape.d_model
sess = eng.new_session(B, (torch.randn(B * T, d, device=dev) * 0.5).bfloat16())
sess.ids.random_(0, 50000)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for q in (4, 1):
    plans = sess._step_plans(q)
    def run():
        sess.cur_len.fill_(q if q > 1 else 8)
        sess._run(plans)
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.graph(g, stream=side):
        run()
    torch.cuda.current_stream().wait_stream(side)
    g.replay()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(10):
        g.replay()
    e1.record()
    e1.synchronize()
    print(f"q={q}: {e0.elapsed_time(e1) / 10:.3f} ms", flush=True)

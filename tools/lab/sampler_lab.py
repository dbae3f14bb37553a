"""Greedy sampler step time at B = 32, V = 51866: with / without timestamps (development)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kotoba-whisper_amd"))
import torch  # noqa: E402

from kwhisper import ops  # noqa: E402
from kwhisper.config import LARGE_V3, generation_constants  # noqa: E402

gen = generation_constants(LARGE_V3)
B, V, P = 32, LARGE_V3.vocab_size, 3
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for rt in (False, True):
    ids = torch.zeros((B, 449), dtype=torch.int64, device="cuda")
    ids[:, :P] = torch.tensor([50258, 50266, 50360])
    ids[:, P:60] = torch.randint(0, 50000, (B, 60 - P))
    cur = torch.tensor([60], dtype=torch.int32, device="cuda")
    unf = torch.ones(B, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    nun = torch.zeros(1, dtype=torch.int32, device="cuda")
    sup = torch.zeros(V, dtype=torch.uint8, device="cuda")
    lg = torch.randn(B, V, device="cuda")
    ws = torch.zeros(ops.greedy_step_workspace_bytes(B) // 4 + 1, device="cuda")
    plan = ops.SamplerPlan(lg, sup, None, ids, cur, unf, cnt, nun, return_timestamps=rt, ts_begin=gen.timestamp_begin,
                           no_ts_id=gen.no_timestamps_token_id, eos_id=gen.eos_token_id, pad_id=gen.pad_token_id,
                           max_initial_ts=gen.max_initial_timestamp_index, max_length=448, begin_index=P, workspace=ws)

    def step():
        cur.fill_(60)
        plan()

    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.graph(g, stream=side):
        for _ in range(20):
            step()
    torch.cuda.current_stream().wait_stream(side)
    g.replay()
    torch.cuda.synchronize()
    e0.record()
    g.replay()
    e1.record()
    e1.synchronize()
    print(f"return_timestamps={rt}: {e0.elapsed_time(e1) * 1e3 / 20:.1f} us per step (incl. a cur_len fill)", flush=True)

#!/usr/bin/env python
"""Lab (r03): can a B = 16 half-batch's latency-bound chain (the decode linears + self-attention) run beside
the other half's HBM-bound cross-attention K/V stream?  Graph-replayed, large-v3 bf16, random weights.

  chain(X) = embed + per layer [qkv, self, o, xq, xo, fc1, fc2] + LM head of half X   (no cross-attention)
  cross(X) = the 32 cross-attention launches of half X

Each graph is captured alone on its stream; concurrency = replaying graphs on different streams at once
(the hardware interleaves them).  A one-graph fork/join capture checks whether a single graph's parallel
branches run concurrently too.  Prints ms per replay set."""
import json
import os
import sys
import time

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
T, d = shape.max_source_positions, shape.d_model
HALF = int(os.environ.get("LAB_HALF", "16"))


def session(B):
    enc = (torch.randn(B * T, d, device=dev) * 0.5).bfloat16()
    s = eng.new_session(B, enc)
    s.ids.random_(0, 50000)
    s.cur_len.fill_(64)
    return s


def tag(p):
    return p[0] if isinstance(p, tuple) else getattr(p, "tag", "linear")


def parts(s):
    seq = s._step_plans(1)
    return [p for p in seq if tag(p) != "cross"], [p for p in seq if tag(p) == "cross"]


def capture(fns, stream):
    g = torch.cuda.CUDAGraph()
    stream.wait_stream(torch.cuda.current_stream())
    with torch.cuda.graph(g, stream=stream):
        for f in fns:
            f()
    torch.cuda.current_stream().wait_stream(stream)
    return g


full = session(2 * HALF)
A, B = session(HALF), session(HALF)
streams = [torch.cuda.Stream() for _ in range(4)]
cur = torch.cuda.current_stream()
chA, crA = parts(A)
chB, crB = parts(B)
g_full = capture([lambda: full._run(full._step_plans(1))], streams[0])
g_chA = capture([lambda: A._run(chA)], streams[0])
g_crA = capture([lambda: A._run(crA)], streams[1])
g_chB = capture([lambda: B._run(chB)], streams[2])
g_crB = capture([lambda: B._run(crB)], streams[3])
g_stepA = capture([lambda: A._run(A._step_plans(1))], streams[0])


def forkjoin():
    """ONE graph: chain(A) on one stream, cross(B) on another, forked from / joined to the capture stream."""
    g = torch.cuda.CUDAGraph()
    s0, s1 = streams[0], streams[1]
    s0.wait_stream(cur)
    with torch.cuda.graph(g, stream=s0):
        s1.wait_stream(s0)
        A._run(chA)
        with torch.cuda.stream(s1):
            B._run(crB)
        s0.wait_stream(s1)
    cur.wait_stream(s0)
    return g


g_fj = forkjoin()
torch.cuda.synchronize()
res = {}


def bench(name, graphs, n=30):
    def run():
        for i, g in enumerate(graphs):
            st = streams[i]
            st.wait_stream(cur)
            with torch.cuda.stream(st):
                g.replay()
        for i in range(len(graphs)):
            cur.wait_stream(streams[i])

    for _ in range(3):
        run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        run()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / n * 1e3
    res[name] = round(ms, 3)
    print(f"{name:52s} {ms:7.3f} ms", flush=True)


bench(f"full step B={2 * HALF}", [g_full])
bench(f"half step B={HALF}", [g_stepA])
bench("chain(A) alone", [g_chA])
bench("cross(A) alone", [g_crA])
bench("chain(A) | cross(B) on 2 streams", [g_chA, g_crB])
bench("chain(A) | chain(B) on 2 streams", [g_chA, g_chB])
bench("cross(A) | cross(B) on 2 streams", [g_crA, g_crB])
bench("chain(A) | cross(A) | chain(B) | cross(B) 4 streams", [g_chA, g_crA, g_chB, g_crB])
bench("fork/join graph: chain(A) || cross(B)", [g_fj])
print(json.dumps(res))

#!/usr/bin/env python
"""Lab (r04): two B = 32 batches decoding at once on one GPU -- does batch B's latency-bound linear chain run
beside batch A's HBM-bound cross-attention stream well enough to raise throughput?

Each batch is its own DecodeSession (production step: fused self / cross blocks, bf16 large-v3, random weights),
its one-step graph captured on its own stream.  Timed (ms per step, per batch):
  one        one session's graph replayed N times
  two-free   both sessions' graphs replayed N times each on two streams, no ordering between them
  two-layer  ONE graph: both sessions' steps with their layers interleaved across two streams -- session B's
             layer l runs on stream 1 after A's layer l has started (A's cross-attention beside B's chain).
Throughput gain = 2 x one / two."""
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
B = int(os.environ.get("LAB_B", "32"))
N = int(os.environ.get("LAB_N", "40"))


def session():
    enc = (torch.randn(B * T, d, device=dev) * 0.5).bfloat16()
    s = eng.new_session(B, enc)
    s.ids.random_(0, 50000)
    s.cur_len.fill_(64)
    return s


def capture(fn, stream):
    g = torch.cuda.CUDAGraph()
    stream.wait_stream(torch.cuda.current_stream())
    with torch.cuda.graph(g, stream=stream):
        fn()
    torch.cuda.current_stream().wait_stream(stream)
    return g


A, Bs = session(), session()
sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
cur = torch.cuda.current_stream()
plan_a, plan_b = A._step_plans(1, fused=True), Bs._step_plans(1, fused=True)
g_a = capture(lambda: A._run(plan_a), sa)
g_b = capture(lambda: Bs._run(plan_b), sb)


def layers(plan):
    """The step plan cut into [embed] + one list per decoder layer + [LM head]."""
    head, body, tail = plan[:1], plan[1:-1], plan[-1:]
    per = len(body) // shape.decoder_layers
    return [head] + [body[i * per:(i + 1) * per] for i in range(shape.decoder_layers)] + [tail]


def interleaved():
    la, lb = layers(plan_a), layers(plan_b)
    g = torch.cuda.CUDAGraph()
    sa.wait_stream(cur)
    with torch.cuda.graph(g, stream=sa):
        sb.wait_stream(sa)
        for i in range(len(la)):
            A._run(la[i])
            ev = torch.cuda.Event()
            ev.record(sa)
            with torch.cuda.stream(sb):
                sb.wait_event(ev)  # B's layer i starts once A's layer i is issued ahead of it
                Bs._run(lb[i])
        sa.wait_stream(sb)
    cur.wait_stream(sa)
    return g


g_il = interleaved()
res = {}


def bench(name, fn, steps_per_call):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(N):
        fn()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / N * 1e3 / steps_per_call
    res[name] = round(ms, 4)
    print(f"{name:44s} {ms:8.4f} ms per batch-step", flush=True)


def one():
    g_a.replay()


def two_free():
    sa.wait_stream(cur)
    sb.wait_stream(cur)
    with torch.cuda.stream(sa):
        g_a.replay()
    with torch.cuda.stream(sb):
        g_b.replay()
    cur.wait_stream(sa)
    cur.wait_stream(sb)


def two_layer():
    g_il.replay()


def masked_stream(bits):
    """A HIP stream restricted to the CUs whose bits are set (hipExtStreamCreateWithCUMask through ctypes on the
    HIP runtime torch has loaded), wrapped for torch."""
    import ctypes

    hip = ctypes.CDLL("libamdhip64.so")
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    words = (ncu + 31) // 32
    mask = (ctypes.c_uint32 * words)()
    for c in range(ncu):
        if bits(c):
            mask[c // 32] |= 1 << (c % 32)
    st = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(st), ctypes.c_uint32(words), mask)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(st.value)


ncu = torch.cuda.get_device_properties(0).multi_processor_count
masks = {"contiguous halves": (lambda c: c < ncu // 2, lambda c: c >= ncu // 2),
         "even / odd CUs": (lambda c: c % 2 == 0, lambda c: c % 2 == 1)}
masked = {}
for name, (ma, mb) in masks.items():
    ms_a, ms_b = masked_stream(ma), masked_stream(mb)

    def run(ms_a=ms_a, ms_b=ms_b):
        ms_a.wait_stream(cur)
        ms_b.wait_stream(cur)
        with torch.cuda.stream(ms_a):
            g_a.replay()
        with torch.cuda.stream(ms_b):
            g_b.replay()
        cur.wait_stream(ms_a)
        cur.wait_stream(ms_b)

    def run_one(ms_a=ms_a):
        ms_a.wait_stream(cur)
        with torch.cuda.stream(ms_a):
            g_a.replay()
        cur.wait_stream(ms_a)

    masked[name] = (run, run_one)

bench("one session", one, 1)
bench("two sessions, free-running streams", two_free, 2)
bench("two sessions, layer-interleaved graph", two_layer, 2)
for name, (run, run_one) in masked.items():
    bench(f"one session on half the CUs ({name})", run_one, 1)
    bench(f"two sessions, CU-masked ({name})", run, 2)
bench("one session (again)", one, 1)
res["gain_free"] = round(res["one session"] / res["two sessions, free-running streams"], 4)
res["gain_layer"] = round(res["one session"] / res["two sessions, layer-interleaved graph"], 4)
print(json.dumps(res), flush=True)

"""Split-batch decode experiment (development): one B=32 decode step vs two B=16 half steps, run back
to back on one stream or concurrently on two streams (each half its own hipGraph)."""
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


def session(B):
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


full = session(32)
ha, hb = session(16), session(16)
sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
gf = capture(lambda: full._run(full._step_plans(1)), sa)
ga = capture(lambda: ha._run(ha._step_plans(1)), sa)
gb = capture(lambda: hb._run(hb._step_plans(1)), sb)
torch.cuda.synchronize()


def bench(name, fn, n=40):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    print(f"{name:44s} {(time.perf_counter() - t0) / n * 1e3:7.3f} ms/step", flush=True)


cur = torch.cuda.current_stream()


def both_serial():
    ga.replay()
    gb.replay()


def both_concurrent():
    sa.wait_stream(cur)
    sb.wait_stream(cur)
    with torch.cuda.stream(sa):
        ga.replay()
    with torch.cuda.stream(sb):
        gb.replay()
    cur.wait_stream(sa)
    cur.wait_stream(sb)


bench("B=32 one graph", gf.replay)
bench("B=16 one half", ga.replay)
bench("two halves, one stream", both_serial)
bench("two halves, two streams (concurrent)", both_concurrent)

# CU-masked streams: each half on its own half of the chip (kw_stream_create_cu_range)
from kwhisper import ops  # noqa: E402

ncu = torch.cuda.get_device_properties(0).multi_processor_count
for split in (ncu // 2, (ncu * 5) // 8):
    ma, mb = ops.cu_range_stream(0, split), ops.cu_range_stream(split, ncu)
    gma = capture(lambda: ha._run(ha._step_plans(1)), ma)
    gmb = capture(lambda: hb._run(hb._step_plans(1)), mb)
    torch.cuda.synchronize()

    def masked():
        ma.wait_stream(cur)
        mb.wait_stream(cur)
        with torch.cuda.stream(ma):
            gma.replay()
        with torch.cuda.stream(mb):
            gmb.replay()
        cur.wait_stream(ma)
        cur.wait_stream(mb)

    def masked_a():
        ma.wait_stream(cur)
        with torch.cuda.stream(ma):
            gma.replay()
        cur.wait_stream(ma)

    bench(f"B=16 half alone on CUs [0,{split})", masked_a)
    bench(f"two halves, CU-masked {split}/{ncu - split}", masked)

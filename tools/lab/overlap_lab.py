"""Encoder / decode overlap experiment (development): can the next batch's encoder (MFMA-bound) run on
a CU-masked stream while this batch's latency-bound decode steps replay on the rest of the chip?

Times, for large-v3 at B = 32: 128 graph-replayed decode steps alone, encoder + cross-K/V alone, and
both at once, for several CU splits (hipExtStreamCreateWithCUMask; mask bit i = CU i).
"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kotoba-whisper_amd"))
import torch  # noqa: E402

from kwhisper.config import PRESETS  # noqa: E402
from kwhisper.engine import WhisperEngine  # noqa: E402
from kwhisper.synthetic import synthetic_state_dict_torch  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
dev = torch.device("cuda")
NCU = torch.cuda.get_device_properties(0).multi_processor_count


def masked_stream(bits):
    words = (ctypes.c_uint32 * ((NCU + 31) // 32))()
    for b in bits:
        words[b // 32] |= 1 << (b % 32)
    h = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), ctypes.c_uint32(len(words)), words)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(h.value)


shape = PRESETS["large-v3"]
sd = synthetic_state_dict_torch(shape, seed=0, device=dev)
eng = WhisperEngine(shape, sd, dtype=torch.bfloat16, device=dev)
del sd
T, d, B = shape.max_source_positions, shape.d_model, 32
enc = (torch.randn(B * T, d, device=dev) * 0.5).bfloat16()
sess = eng.new_session(B, enc)
sess.ids.random_(0, 50000)
feats = torch.randn(B, shape.num_mel_bins, 3000, device=dev)
cross2 = torch.empty_like(sess.cross)
NSTEP = int(os.environ.get("NSTEP", "128"))


def capture(stream):
    g = torch.cuda.CUDAGraph()
    stream.wait_stream(torch.cuda.current_stream())
    with torch.cuda.graph(g, stream=stream):
        sess._run(sess._step_plans(1))
    torch.cuda.current_stream().wait_stream(stream)
    return g


def decode(g, stream):
    with torch.cuda.stream(stream):
        sess.cur_len.fill_(8)
        for _ in range(NSTEP):
            g.replay()


def encoder(stream):
    with torch.cuda.stream(stream):
        h = eng.encode(feats)
        eng.cross_kv(h, B, out=cross2)


def run(name, fns):
    torch.cuda.synchronize()
    for _ in range(2):
        for f in fns:
            f()
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for f in fns:
        f()
    torch.cuda.synchronize()
    print(f"{name:60s} {(time.perf_counter() - t0) * 1e3:8.1f} ms", flush=True)


full = torch.cuda.Stream()
hi = torch.cuda.Stream(priority=-1)
g_full = capture(full)
g_hi = capture(hi)
run("decode x%d alone (full chip)" % NSTEP, [lambda: decode(g_full, full)])
run("encoder + cross-KV alone (full chip)", [lambda: encoder(full)])
run("serial: encoder then decode (full chip)", [lambda: encoder(full), lambda: decode(g_full, full)])
plain = torch.cuda.Stream()
run("encoder (plain stream) + decode (high-priority stream)", [lambda: encoder(plain), lambda: decode(g_hi, hi)])
for n_enc in (64, 96, 128, 160):
    se = masked_stream(range(n_enc))
    run(f"[low {n_enc} CUs] encoder alone (masked)", [lambda: encoder(se)])
    run(f"[low {n_enc} CUs] both, decode full chip", [lambda: encoder(se), lambda: decode(g_full, full)])
    run(f"[low {n_enc} CUs] both, decode full chip high priority", [lambda: encoder(se), lambda: decode(g_hi, hi)])

"""r03ag lab: the large-v3 encoder at B = 32 as ONE pass vs two B = 16 halves issued interleaved on two streams
(each GEMM's last round of tiles leaves CUs idle -- QKV 11.02, out / fc2 3.67, fc1 14.69 rounds of 256 tiles --
which the other half's kernels could fill).  Bitwise check of the halves against the full pass, then timing
(HIP events, 6 alternating rounds)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kotoba-whisper_amd"))
import torch  # noqa: E402

from kwhisper import ops  # noqa: E402
from kwhisper.config import PRESETS  # noqa: E402
from kwhisper.engine import _EncoderBuffers, _HD  # noqa: E402
from kwhisper.generation import KWhisperForConditionalGeneration  # noqa: E402
from kwhisper.synthetic import synthetic_state_dict_torch  # noqa: E402

dev = torch.device("cuda")
shape = PRESETS["large-v3"]
sd = synthetic_state_dict_torch(shape, seed=0, device=dev)
model = KWhisperForConditionalGeneration.from_state_dict(shape, sd, dtype=torch.bfloat16, device=dev)
del sd
torch.cuda.empty_cache()
eng = model.engine
s = eng.shape
B, T = 32, s.max_source_positions
mel = torch.randn(B, s.num_mel_bins, s.n_frames, device=dev) * 0.5

full = eng.encoder_buffers(B)
halves = [_EncoderBuffers(eng, B // 2), _EncoderBuffers(eng, B // 2)]
streams = [torch.cuda.Stream(), torch.cuda.Stream()]


def run_plan(p, Bh):
    if isinstance(p, tuple):
        if p[0] == "ln":
            ops.layernorm(p[1], p[2], p[3], s.layer_norm_eps, p[4], delta=p[5])
        else:
            ops.attention(p[1], Bh, eng.H, T, _HD, p[2], q_log2=p[3])
    else:
        p()


def split_encode():
    cur = torch.cuda.current_stream()
    for i, st in enumerate(streams):
        st.wait_stream(cur)
        with torch.cuda.stream(st):
            ops.mel_to_time_major(mel[i * 16:(i + 1) * 16].contiguous(), eng.c_pad, eng.dtype, out=halves[i].mel_tm)
    for j in range(len(full.plans)):
        for i, st in enumerate(streams):
            with torch.cuda.stream(st):
                run_plan(halves[i].plans[j], B // 2)
    for st in streams:
        cur.wait_stream(st)


ref = eng.encode(mel).clone()
split_encode()
torch.cuda.synchronize()
got = torch.cat([halves[0].out, halves[1].out])
print("bitwise equal to the one-pass encoder:", torch.equal(ref.view(torch.int16), got.view(torch.int16)), flush=True)

best = {}
for name, fn in [("one pass B=32", lambda: eng.encode(mel)), ("two B=16 halves, 2 streams", split_encode)] * 6:
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        fn()
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / 3
    print(f"{name:28s} {ms:8.2f} ms", flush=True)
    best[name] = min(best.get(name, 1e9), ms)
print({k: round(v, 2) for k, v in best.items()})

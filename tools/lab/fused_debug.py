"""Debug: the fused QKV+self launch vs the two-launch plan inside the tiny bf16 engine, step by step (layer 0)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "kotoba-whisper_amd"), os.path.join(ROOT, "tests"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from kwhisper.config import TINY, generation_constants  # noqa: E402
from kwhisper.engine import WhisperEngine  # noqa: E402
from kwhisper.synthetic import synthetic_state_dict  # noqa: E402
from _util import oracle_features  # noqa: E402

g = dict(np.load(os.path.join(ROOT, "tests/golden/tiny_fp32.npz")))
feats = torch.from_numpy(oracle_features(TINY, g["cases"])).cuda()
sd = synthetic_state_dict(TINY, 0)
ef = WhisperEngine(TINY, sd, dtype=torch.bfloat16, generation_config=generation_constants(TINY), fuse_qkv_self=True)
ep = WhisperEngine(TINY, sd, dtype=torch.bfloat16, generation_config=generation_constants(TINY), fuse_qkv_self=False)
enc = ep.encode(feats)
sf, sp = ef.new_session(4, enc), ep.new_session(4, enc)
seq = torch.from_numpy(g["greedy_sequences"])[:, :-1].cuda()
P, T = 4, seq.shape[1]
for s in (sf, sp):
    s.ids.zero_()
    s.ids[:, :T].copy_(seq)
    s.cur_len.fill_(P)
    s._run(s._step_plans(P))
torch.cuda.synchronize()
print("prefill caches equal", torch.equal(sf.kc, sp.kc), torch.equal(sf.vc, sp.vc))
stf, stp = sf._step_plans(1, fused=True), sp._step_plans(1, fused=False)
print("plan tags", [getattr(p, "tag", p[0] if isinstance(p, tuple) else "?") for p in stf[:4]],
      [getattr(p, "tag", p[0] if isinstance(p, tuple) else "?") for p in stp[:4]])
bf, bp_ = sf._buffers(1), sp._buffers(1)
for t in range(P, T):
    for s in (sf, sp):
        s.cur_len.fill_(t + 1)
    # layer 0 only: embed + fused  vs  embed + qkv + self
    sf._run(stf[:2])
    sp._run(stp[:3])
    torch.cuda.synchronize()
    a, b = bf["attn"].float(), bp_["attn"].float()
    q = bp_["qkv"][:, :384].float().view(4, 6, 1, 64)
    L = t + 1
    k = sp.kc[0, :, :, :L].float()
    v = sp.vc[0, :, :, :L].float()
    ref = (torch.softmax(q @ k.transpose(-1, -2), -1) @ v).view(4, 384)
    print(f"t={t} L={L} hb equal {torch.equal(bf['hb'], bp_['hb'])} kc0 equal {torch.equal(sf.kc[0], sp.kc[0])} "
          f"vc0 equal {torch.equal(sf.vc[0], sp.vc[0])} attn diff {(a - b).abs().max().item():.4g} "
          f"fused-ref {(a - ref).abs().max().item():.4g} plain-ref {(b - ref).abs().max().item():.4g} "
          f"ws {int(sf.qs_ws.view(torch.int32).abs().sum())}", flush=True)
    # now the rest of the step on both, from the plain attention output so the two stay in lockstep
    bf["attn"].copy_(bp_["attn"])
    sf._run(stf[2:])
    sp._run(stp[3:])
    torch.cuda.synchronize()
    print("   logits diff after the full step", (sf.logits - sp.logits).abs().max().item(),
          "caches equal", torch.equal(sf.kc, sp.kc), torch.equal(sf.vc, sp.vc), flush=True)

# teacher-forced end to end (no lockstep): both engines vs the fp32 reference's top-8 logits
seqc = torch.from_numpy(g["greedy_sequences"])
lf = ef.new_session(4, enc).teacher_forced_logits(seqc[:, :-1], 4).float().cpu().numpy()
lp = ep.new_session(4, enc).teacher_forced_logits(seqc[:, :-1], 4).float().cpu().numpy()
idx, val = g["greedy_logits_top_idx"].astype(np.int64), g["greedy_logits_top_val"]
n = idx.shape[1]
for name, lg in (("fused", lf), ("plain", lp)):
    got = np.take_along_axis(lg[:, :n], idx, axis=-1)
    e = np.abs(got - val)
    print(f"{name}: top-8 vs fp32 max {e.max():.4f} mean {e.mean():.4f}; per-step max", np.round(e.max((0, 2)), 3).tolist())
d = np.abs(lf - lp)
print("fused vs plain full-vocab: max", d.max(), "mean", d.mean(), "per-step mean", np.round(d.mean((0, 2)), 3).tolist())

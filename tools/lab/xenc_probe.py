"""Diagnostics for kw_cross_attn_enc (lab): error patterns per query / channel slice for a few probes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kotoba-whisper_amd")]
import torch  # noqa: E402

from kwhisper import ops  # noqa: E402


def run(B, S, D, H, q_len, u_scale, zero_u=False):
    torch.manual_seed(0)
    enc = torch.randn(B, S, D, device="cuda").bfloat16()
    u = (torch.randn(B * q_len, H, D, device="cuda") * (u_scale / D ** 0.5)).bfloat16()
    if zero_u:
        u.zero_()
    z = torch.zeros(B * q_len, H * D, device="cuda", dtype=torch.bfloat16)
    ws = torch.zeros((ops.cross_attn_enc_workspace_bytes(B, D) + 3) // 4, device="cuda")
    ops.cross_attn_enc(enc, B, S, D, u, q_len, H, z, ws)
    torch.cuda.synchronize()
    e = enc.float()
    uu = u.float().view(B, q_len * H, D)
    p = torch.softmax(uu @ e.transpose(1, 2), -1)
    ref = (p @ e).view(B * q_len, H, D)
    zz = z.float().view_as(ref)
    err = (zz - ref).abs()
    print(f"B={B} S={S} D={D} H={H} q={q_len} u_scale={u_scale} zero_u={zero_u}: max err {err.max():.4g} "
          f"mean {err.mean():.4g} max|ref| {ref.abs().max():.3g}")
    print("  per query max err:", [round(x, 3) for x in err.amax(dim=(0, 2)).tolist()])
    nw = 8 if D % 256 == 0 else 4
    print("  per wave-slice max err:", [round(x, 3) for x in err.view(B * q_len, H, nw, -1).amax(dim=(0, 1, 3)).tolist()])
    print("  per 16-channel block (first slice):", [round(x, 3) for x in err[..., : D // nw].reshape(B * q_len, H, -1, 16).amax(dim=(0, 1, 3)).tolist()])
    print("  z[0,0,:8]", zz[0, 0, :8].tolist())
    print("  ref[0,0,:8]", ref[0, 0, :8].tolist())
    hdr = ws.view(torch.int32)[: 2 * B + 1]
    print("  header nonzero:", int((hdr != 0).sum()))


if __name__ == "__main__":
    run(2, 1500, 1280, 20, 1, 3.0, zero_u=True)
    run(2, 1500, 1280, 20, 1, 0.0)
    run(300, 64, 1280, 20, 1, 3.0)
    run(2, 1500, 1280, 20, 1, 3.0)
    run(2, 1500, 384, 6, 1, 3.0)

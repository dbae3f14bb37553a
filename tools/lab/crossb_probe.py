#!/usr/bin/env python
"""Cross-attention stream vs batch size (lab r05r): is cross_attn_row_kernel bound by HBM (time ~ B) or by the
per-CU stream of the CUs holding the most (row, head) pairs (time ~ ceil(B * H / CUs))?  Times ops.cross_attn_step
(the row kernel for B * H in [CUs, 3 CUs]) over 32 distinct K/V buffers in a captured graph, as tools/kbench.py does.
"""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kotoba-whisper_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

from kwhisper import ops  # noqa: E402
from kbench import timeit  # noqa: E402


def main():
    dev = torch.device("cuda")
    H, S, nl = 20, 1500, 32
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    res = {"cus": ncu}
    for B in [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "13,20,25,26,29,32,35,38").split(",")]:
        q = torch.randn(B, H * 64, device=dev).bfloat16()
        out = torch.empty(B, H * 64, device=dev).bfloat16()
        cross = [torch.randn(2, B, H, S, 64, device=dev).bfloat16() for _ in range(nl)]
        ws = torch.zeros(ops.cross_attn_workspace_bytes(B, 1, H, 64, S) // 4 + 1, device=dev)
        fns = [lambda c=c: ops.cross_attn_step(q, B, 1, H, 64, c[0], c[1], S, out, ws) for c in cross]
        us = timeit(fns, 20)
        pairs = B * H
        res[B] = {"us": round(us, 2), "TBps": round(2 * B * H * S * 64 * 2 / us / 1e6, 3), "pairs": pairs,
                  "max_pairs_per_cu": -(-pairs // ncu), "row_kernel": ops.cross_attn_pair_kernel(B * H, S)}
        del cross, ws
        torch.cuda.empty_cache()
        print(json.dumps({B: res[B]}), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()

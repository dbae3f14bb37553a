"""The decode kernels issue their loads back to back (CPU check of the gfx950 device assembly).

Each kernel below is written to put every load of its memory round trip in flight before the first
wait.  A compiler-placed ``s_waitcnt vmcnt(0)`` between those loads (an address that depends on a load,
a phi between a loaded register and a constant) serialises them: round 2 measured 8.7 -> 5.7 us for the
self-attention at t = 68 and a 2-3 % faster decode step once three such waits were gone
(profiles/r02k_lab_notes.md).  The counts are the loads each kernel issues before its first vmcnt(0).
"""
from __future__ import annotations

import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import isa_scan  # noqa: E402

pytestmark = pytest.mark.skipif(not os.path.exists(isa_scan.HIPCC) and not shutil.which("hipcc"),
                                reason="hipcc not available")

CASES = {
    "attention.hip": [
        # q row + 8 K + 8 V rows (+ the cache append of split 0); the beam instantiation adds its 8 slot rows
        (r"self_attn_step1ItLb0E", 19),
        (r"self_attn_step1ItLb1E", 27),
        (r"cross_attn_dma_kernel", 17),
        (r"cross_attn_multi_kernelItLi4E", 20),  # 4 query rows + 8 K + 8 V rows
        (r"cross_attn_mfma_kernel", 20),
    ],
    "sampling.hip": [
        (r"greedy_step_split_kernel", 33),  # 16 logits + 16 SuppressTokens bytes (+ cur_len)
        (r"greedy_step_split_ts_kernel", 33),
    ],
    "beam.hip": [(r"beam_logprobs_split_kernel", 33)],
    # the LM head's run: epilogue constants + 10 activation fragments + two groups' weights + every prefetch of the
    # group loop before any vmcnt(0) (r05: the loop's joins no longer drain the prefetch)
    # (r06: the same run with the greedy step's mask bytes and cur_len beside the constants -- kw_dec_lm_greedy)
    "declin.hip": [(r"lm_head_kernelILb0E", 50), (r"lm_head_kernelILb1E", 50)],
}


@pytest.fixture(scope="module")
def asm():
    cache = {}

    def get(f):
        if f not in cache:
            cache[f] = isa_scan.device_asm(os.path.join(isa_scan.CSRC, f))
        return cache[f]

    return get


@pytest.mark.parametrize("src,pattern,n", [(f, p, n) for f, cs in CASES.items() for p, n in cs])
def test_loads_in_flight_before_first_wait(asm, src, pattern, n):
    got = isa_scan.leading_loads(asm(src), pattern)
    assert got >= n, f"{pattern}: {got} loads before the first vmcnt(0), expected >= {n}"

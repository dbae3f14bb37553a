#!/usr/bin/env python
"""Load-issue scan of the gfx950 device assembly (development tool and CPU regression check).

A kernel that is meant to put all its loads in flight at once (one memory round trip) loses that the
moment the compiler places an ``s_waitcnt vmcnt(0)`` between two of them: an address computed from a
loaded value, a phi between a loaded register and a constant, or a load inside a branch whose join needs
the value.  Round 2 found three such cases on the decode path (profiles/r02k_lab_notes.md): the beam
slot-table lookup inside the self-attention's K/V addresses (16 serialised row loads, also on the greedy
path), the SuppressTokens byte loaded inside the samplers' per-element compare chain, and the LM head's
epilogue constants loaded behind the next group's weight prefetch.

    python tools/isa_scan.py [file.hip ...]       # every kernel: its load / vmcnt(0) / barrier sequence

``leading_loads(asm, symbol)`` counts the loads a kernel issues, in text order, before its first
``s_waitcnt vmcnt(0)`` (tests/test_isa_scan.py holds the decode kernels to their intended counts).
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "kotoba-whisper_amd", "csrc")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
_LOAD = re.compile(r"^(global|buffer|flat)_load")


def device_asm(hip_file: str) -> str:
    """gfx950 device assembly of one source file (hipcc --cuda-device-only -S, the Makefile's flags)."""
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "k.s")
        subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "-munsafe-fp-atomics",
                        "--cuda-device-only", "-S", "-o", out, hip_file], check=True,
                       stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        with open(out) as f:
            return f.read()


def kernels(asm: str) -> dict[str, list[str]]:
    """symbol -> its instruction lines (text order)."""
    lines = asm.split("\n")
    starts = [(i, ln.split(":")[0]) for i, ln in enumerate(lines) if re.match(r"^_Z\S*:", ln)]
    out = {}
    for n, (i, name) in enumerate(starts):
        end = starts[n + 1][0] if n + 1 < len(starts) else len(lines)
        out[name] = [ln.strip() for ln in lines[i + 1:end]]
    return out


def sequence(body: list[str]) -> list[str]:
    """L = load (Ln: non-temporal), W0 = s_waitcnt vmcnt(0), B = s_barrier, E = s_endpgm."""
    seq = []
    for t in body:
        if _LOAD.match(t):
            seq.append("Ln" if " nt" in t else "L")
        elif t.startswith("s_waitcnt") and "vmcnt(0)" in t:
            seq.append("W0")
        elif t.startswith("s_barrier"):
            seq.append("B")
        elif t.startswith("s_endpgm"):
            seq.append("E")
    return seq


def find(asm: str, pattern: str) -> tuple[str, list[str]]:
    ks = {k: v for k, v in kernels(asm).items() if re.search(pattern, k)}
    if len(ks) != 1:
        raise KeyError(f"{pattern!r} matches {sorted(ks)}")
    return next(iter(ks.items()))


def leading_loads(asm: str, pattern: str) -> int:
    """Loads issued (text order) before the kernel's first vmcnt(0)."""
    n = 0
    for tok in sequence(find(asm, pattern)[1]):
        if tok == "W0":
            break
        if tok.startswith("L"):
            n += 1
    return n


def main(argv: list[str]) -> None:
    files = argv or [os.path.join(CSRC, f) for f in sorted(os.listdir(CSRC)) if f.endswith(".hip")]
    for f in files:
        for name, body in kernels(device_asm(f)).items():
            print(os.path.basename(f), name[:70], "|", " ".join(sequence(body))[:300])


if __name__ == "__main__":
    main(sys.argv[1:])

#!/usr/bin/env python
"""r04: does a HIP event cover a 4-byte non_blocking device -> pinned-host copy queued before it?

decode.py's stop poll copies the device unfinished-row count into a pinned slot, records an event on the same
(current) stream, and reads the slot after the event completes.  r03al saw a FRESH pinned buffer read 0 once
(an early stop).  This reproduces the pattern in isolation with a value the host can check: the device word is
set by a kernel queued behind a spin kernel (so the copy is genuinely in flight when the event is recorded),
then copied, evented, synchronized and read.  Variants:
  fresh    a new pinned tensor per trial (torch.zeros().pin_memory(), the r03al situation)
  reuse    one pinned tensor, sentinel -1 written before each copy (decode.py today)
  blocking torch.cuda.Event(blocking=True)
  stream   the stream synchronized instead of the event
Prints the number of stale reads per variant and the copy's path as torch reports it.
"""
import json
import sys
import time

import torch


def trial(variant, pinned, dev_word, value, spin):
    torch.cuda._sleep(spin)  # keep the stream busy: the fill and the copy queue behind it
    dev_word.fill_(value)
    p = torch.zeros((1,), dtype=torch.int32).pin_memory() if variant == "fresh" else pinned
    if variant != "fresh":
        p[0] = -1
    p.copy_(dev_word, non_blocking=True)
    if variant == "stream":
        torch.cuda.current_stream().synchronize()
    else:
        ev = torch.cuda.Event(blocking=(variant == "blocking"))
        ev.record()
        ev.synchronize()
    return int(p[0]) == value, int(p[0])


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    dev = torch.device("cuda", 0)
    dev_word = torch.zeros((1,), dtype=torch.int32, device=dev)
    pinned = torch.zeros((1,), dtype=torch.int32).pin_memory()
    out = {}
    for variant in ("fresh", "reuse", "blocking", "stream"):
        stale, seen = 0, {}
        t0 = time.time()
        for i in range(n):
            ok, got = trial(variant, pinned, dev_word, 1000 + i, spin=20000 if i % 2 else 0)
            if not ok:
                stale += 1
                seen[got] = seen.get(got, 0) + 1
        out[variant] = {"trials": n, "stale": stale, "stale_values": dict(list(seen.items())[:8]),
                        "seconds": round(time.time() - t0, 2)}
        print(variant, out[variant], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()

#!/usr/bin/env python
"""r04: is a non_blocking device -> pinned copy queued right after a hipGraph replay ordered
after the graph's kernels?  decode.py copies the unfinished-row count the step graph's sampler writes; r03al saw a
fresh session read 0 (the count's initial value) and stop early.  tools/lab/pinned_lab.py found the copy ordered
after a plain kernel (0 stale reads in 8,000 trials); this repeats the check with the writer INSIDE a replayed
graph (a spin kernel, then an increment), the decode loop's pattern:

  graph   = [spin(cycles), word += 1]         captured once on a side stream
  trial   : pinned[0] = -1; graph.replay() x K; pinned.copy_(word, non_blocking=True); event; sync; check
Variants: K = 1 / 2 replays per copy, a fresh zero-filled pinned tensor per trial, and the event replaced by a stream
synchronize.  A read of -1 or a value behind the expected count means the copy overtook the graph."""
import json
import sys

import torch


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
    dev = torch.device("cuda", 0)
    word = torch.zeros((1,), dtype=torch.int32, device=dev)
    side = torch.cuda.Stream()
    graphs = {}
    for spin in (0, 20000, 200000):
        g = torch.cuda.CUDAGraph()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.graph(g, stream=side):
            if spin:
                torch.cuda._sleep(spin)
            word.add_(1)
        torch.cuda.current_stream().wait_stream(side)
        graphs[spin] = g
    torch.cuda.synchronize()
    out = {}
    pinned = torch.zeros((1,), dtype=torch.int32).pin_memory()
    for spin, g in graphs.items():
        for k in (1, 2):
            for variant in ("event", "fresh", "stream"):
                stale, seen = 0, {}
                for _ in range(n // 10 if spin == 200000 else n):
                    torch.cuda.synchronize()
                    want = int(word.item()) + k
                    p = torch.zeros((1,), dtype=torch.int32).pin_memory() if variant == "fresh" else pinned
                    if variant != "fresh":
                        p[0] = -1
                    for _ in range(k):
                        g.replay()
                    p.copy_(word, non_blocking=True)
                    if variant == "stream":
                        torch.cuda.current_stream().synchronize()
                    else:
                        ev = torch.cuda.Event()
                        ev.record()
                        ev.synchronize()
                    got = int(p[0])
                    if got != want:
                        stale += 1
                        seen[got - want] = seen.get(got - want, 0) + 1
                key = f"spin{spin}_k{k}_{variant}"
                out[key] = {"stale": stale, "offsets": seen}
                print(key, out[key], flush=True)
        # the r03al loop itself: a fresh zero-filled 5-slot ring, slot = done % 5 with done += 2, the read two
        # replays behind (no sentinel: a stale slot reads 0, the failure r03al saw on slot 4's first use)
        stale, runs = 0, max(1, n // 30)
        for _ in range(runs):
            torch.cuda.synchronize()
            base = int(word.item())
            ring = torch.zeros((5,), dtype=torch.int32).pin_memory()
            events, done = [], 1
            for r in range(10):
                g.replay()
                g.replay()
                done += 2
                slot = done % 5
                ring[slot: slot + 1].copy_(word, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record()
                events.append((ev, slot, base + 2 * (r + 1)))
                if len(events) > 2:
                    e0, s0, want = events.pop(0)
                    e0.synchronize()
                    stale += int(ring[s0]) != want
        out[f"spin{spin}_ring"] = {"stale": stale, "reads": runs * 8}
        print(f"spin{spin}_ring", out[f"spin{spin}_ring"], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()

"""Lab: are the branches of a captured torch.cuda graph (two side streams) co-resident on the GPU?
Build: hipcc -O3 --offload-arch=gfx950 -shared -fPIC tools/lab/graph_lab.hip -o tools/lab/libgraph_lab.so"""
import ctypes
import os
import time

import torch

lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libgraph_lab.so"))
f = torch.zeros(2, dtype=torch.int32, device="cuda")
res = torch.zeros(4, dtype=torch.int64, device="cuda")
ep = torch.zeros(1, dtype=torch.int32, device="cuda")


def launch(which, epoch, s):
    fn = lib.lab_launch_a if which == "a" else lib.lab_launch_b
    assert fn(ctypes.c_void_p(f.data_ptr()), ctypes.c_void_p(res.data_ptr()), epoch,
              ctypes.c_void_p(s.cuda_stream)) == 0


for order in ("ab", "ba"):
    for trial in range(2):
        f.zero_()
        res.zero_()
        torch.cuda.synchronize()
        main = torch.cuda.current_stream()
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        g = torch.cuda.CUDAGraph()
        cap = torch.cuda.Stream()
        cap.wait_stream(main)
        with torch.cuda.graph(g, stream=cap):
            s1.wait_stream(cap)
            s2.wait_stream(cap)
            first, second = (s1, s2)
            with torch.cuda.stream(s1):
                launch(order[0], 1, s1)
            with torch.cuda.stream(s2):
                launch(order[1], 1, s2)
            cap.wait_stream(s1)
            cap.wait_stream(s2)
        main.wait_stream(cap)
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        r = res.cpu().tolist()
        print(f"graph order {order} trial {trial}: A spins {r[0]} B spins {r[1]} (-1 = timeout) "
              f"A ticks {r[2]} B ticks {r[3]} wall {dt * 1e3:.2f} ms", flush=True)
# plain two-stream launches (no graph) for comparison
f.zero_()
res.zero_()
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
torch.cuda.synchronize()
launch("a", 1, s1)
launch("b", 1, s2)
torch.cuda.synchronize()
r = res.cpu().tolist()
print(f"eager two streams: A spins {r[0]} B spins {r[1]} A ticks {r[2]} B ticks {r[3]}", flush=True)

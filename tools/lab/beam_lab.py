"""kw_beam_logprobs timing (development): one-workgroup vs split rows, R running rows, V = 51865."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kotoba-whisper_amd"))
import torch  # noqa: E402

from kwhisper import _lib as L  # noqa: E402
from kwhisper import ops  # noqa: E402

V, P, k = 51865, 3, 10
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
lib = L.load()
for R in (32, 320):
    for rt in (0, 1):
        for split in (False, True):
            ids = torch.randint(0, 50000, (R, 64), device="cuda")
            cur = torch.tensor([20], dtype=torch.int32, device="cuda")
            sup = torch.zeros(V, dtype=torch.uint8, device="cuda")
            done = torch.zeros(1, dtype=torch.int32, device="cuda")
            lg = torch.randn(R, V, device="cuda") * 3
            cv = torch.empty((R, k), device="cuda")
            ci = torch.empty((R, k), dtype=torch.int32, device="cuda")
            ws = torch.zeros(ops.beam_logprobs_workspace_bytes(R) // 4 + 1, device="cuda") if split else None
            a = L.BeamLogprobsArgs()
            a.logits, a.R, a.V = lg.data_ptr(), R, V
            a.suppress_mask, a.begin_suppress, a.n_begin_suppress = sup.data_ptr(), None, 0
            a.return_timestamps, a.ts_begin, a.no_ts_id, a.eos_id, a.max_initial_ts = rt, 50364, 50363, 50257, 50
            a.ids, a.ids_stride, a.cur_len, a.begin_index, a.k = ids.data_ptr(), 64, cur.data_ptr(), P, k
            a.cand_val, a.cand_idx, a.done = cv.data_ptr(), ci.data_ptr(), done.data_ptr()
            a.workspace = ws.data_ptr() if ws is not None else None
            a.ws_bytes = ws.numel() * 4 if ws is not None else 0
            s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
            for _ in range(3):
                lib.kw_beam_logprobs(ctypes.byref(a), s)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(10):
                lib.kw_beam_logprobs(ctypes.byref(a), s)
            e1.record()
            e1.synchronize()
            print(f"R={R} rt={rt} split={split}: {e0.elapsed_time(e1) * 100:.1f} us", flush=True)

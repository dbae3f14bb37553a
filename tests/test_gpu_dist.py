"""The multi-GPU code path over RCCL on one GPU: bench.py's real rank code and
kwhisper.pseudo_label run under ``torch.distributed.run --nproc-per-node 1`` with the ``nccl`` backend, so
``init_process_group(device_id=...)``, the float64 MAX all_reduce of the step time, the width all_reduce and the
int32 / int64 all_gathers all execute on RCCL (the 8-GPU scaling run is the driver's; gloo world-2 tests cover
the N > 1 host logic on the CPU).  Each run is a child process (started, never exec'd)."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _torchrun(script, *args, timeout=300):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1", "--master-addr=127.0.0.1",
           f"--master-port={port}", script, *args]
    p = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1]
    return json.loads(line)


def test_bench_rank_code_over_rccl():
    """bench.py's rank code (not --stub) under the launcher: the dist path with RCCL at world size 1."""
    r = _torchrun(os.path.join(ROOT, "bench.py"), "--model", "tiny", "--batch", "4", "--steps", "1", "--warmup", "1",
                  "--max-length", "24", "--no-cpu-baseline", "--kernel-iters", "2")
    print("\nbench over RCCL:", json.dumps({k: r[k] for k in ("value", "n_gpus", "dist")}))
    assert r["n_gpus"] == 1 and r["dist"]["backend"] == "nccl" and r["dist"]["ids_gather"]
    assert r["value"] > 0


def test_pseudo_label_over_rccl():
    """pseudo_label's per-round collectives and the deferred exchange, and the ASR pipeline's data-parallel
    gather, over RCCL return the single-process results."""
    r = _torchrun(os.path.join(ROOT, "tests", "_dist_pl.py"))
    print("\npseudo_label over RCCL:", r)
    assert r["backend"] == "nccl" and r["world"] == 1 and r["round"] and r["end"] and r["pipeline"]

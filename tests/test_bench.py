"""bench.py's contract on the CPU: the --gpus N launcher (one rank per GPU under torch.distributed.run, started
as a child process), max-over-ranks timing and the ids gather, in stub mode over gloo; and the kernel-source
hash that ties a committed PMC pass to the kernels it measured."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run_bench(*args, env_extra=None):
    env = dict(os.environ, KW_BENCH_BACKEND="gloo", PYTHONDONTWRITEBYTECODE="1", OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env, capture_output=True,
                       text=True, timeout=240, cwd=ROOT)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


def test_bench_launches_n_ranks_stub():
    """`bench.py --gpus 2` with no launcher environment starts two ranks (reference: accelerate launch
    --multi_gpu, script/distil_whisper_v2.0.sh:26) and prints rank 0's single line with n_gpus 2."""
    r = _run_bench("--gpus", "2", "--stub", "--steps", "2", "--warmup", "1")
    assert r["n_gpus"] == 2 and r["dist"] == {"world": 2, "backend": "gloo"}
    assert r["steps"] == 2 and r["value"] > 0 and r["stub"] is True


def test_bench_single_rank_stub():
    r = _run_bench("--gpus", "1", "--stub", "--steps", "1", "--warmup", "0")
    assert r["n_gpus"] == 1 and r["dist"]["world"] == 1


def test_kernel_source_hash_covers_product_sources_only(tmp_path):
    sys.path.insert(0, ROOT)
    import bench

    files = bench.kernel_source_files()
    names = [os.path.basename(f) for f in files]
    assert "declin.hip" in names and "kwhisper.h" in names and all(os.path.exists(f) for f in files)
    h = bench.kernel_source_hash()
    scratch = os.path.join(ROOT, "kotoba-whisper_amd", "csrc", "_scratch_not_built.hip")
    with open(scratch, "w") as f:
        f.write("// scratch\n")
    try:
        assert bench.kernel_source_hash() == h  # a file outside the Makefile's SRCS does not change it
    finally:
        os.remove(scratch)


def test_pmc_pass_order_by_run_tag():
    """pmc_traffic() reads the newest committed PMC pass: run tags sort by round, then by suffix a..z, aa, ab, ..."""
    sys.path.insert(0, ROOT)
    import bench

    tags = ["r10_x", "r03ad_x", "r01_x", "r03w_x", "r01aa_x", "r01z_x", "r01j_x", "r03_x"]
    assert sorted(tags, key=bench.profile_tag_order) == ["r01_x", "r01j_x", "r01z_x", "r01aa_x", "r03_x", "r03w_x",
                                                          "r03ad_x", "r10_x"]

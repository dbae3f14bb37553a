#!/usr/bin/env python
"""Headline benchmark: audio-seconds/sec of whisper-large-v3 greedy generate, 30 s clips, batch 32/GPU.

One step = one batch of 32 synthetic 30 s clips resident in HBM -> log-mel (HIP) -> encoder ->
cross-attention K/V projection -> greedy decode (4-token prompt, max_length 128 -> 128 new tokens, one hipGraph
replay per step; cross-attention over the per-layer K/V cache, cross_attn_dma_kernel) on the
MI355X engine (bf16).  Weights are random-init of the large-v3 architecture (no checkpoints offline).
N > 1: one process per GPU (torchrun), each rank decodes its own batches (data parallel, weak
scaling), token ids are all-gathered over RCCL at the end (run_pseudo_labelling.py:339-341), and the
time is the max over ranks.

``--gpus N`` without a launcher's WORLD_SIZE starts ``python -m torch.distributed.run --nproc-per-node N`` on
this script as a CHILD process (nothing touches the GPU in the parent) and relays rank 0's line, as the
reference's ``accelerate launch --multi_gpu`` (script/distil_whisper_v2.0.sh:26) starts one process per GPU.

Prints ONE JSON line (rank 0).  Extra fields: ``roofline`` of the decode attention (the cross-attention's
K/V stream, HBM-bound), ``encoder_mfma`` (encoder MFMA fraction), ``decode_kernel_us``
(per-launch time of each decode-step kernel in step context, eager: an upper bound that includes the
dispatch gap; the rocprofv3 trace in profiles/ gives the device times), ``cpu_baseline`` (reference
transformers path on the host cores, bounded sample).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "kotoba-whisper_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
BF16_PEAK_TFLOPS = 2500.0      # dense bf16 MFMA spec
ENC_FLOP_PER_CLIP = 2.2738e12


def kernel_source_files() -> list:
    """The product kernel sources: the ``SRCS`` of csrc/Makefile (what libkwhisper.so is built from), the
    csrc headers they include and include/kwhisper.h.  Read from the Makefile, not globbed, so scratch
    files beside them never change the hash, and no git is needed (the GPU box's snapshot has none)."""
    import re

    csrc = os.path.join(ROOT, "kotoba-whisper_amd", "csrc")
    with open(os.path.join(csrc, "Makefile")) as f:
        m = re.search(r"^SRCS\s*:=\s*(.+)$", f.read(), re.M)
    srcs = m.group(1).split()
    heads = ("kw_common.h", "attn_common.h", "decproj.h", "gemm_common.h", "processors.h")
    return [os.path.join(csrc, x) for x in srcs + list(heads)] + [os.path.join(ROOT, "include", "kwhisper.h")]


def kernel_source_hash() -> str:
    """sha256 over kernel_source_files(): identifies the kernels a PMC pass measured (tools/profile.sh
    stores it beside the counters, on the GPU box; that box-side file is committed as it was written)."""
    import hashlib

    h = hashlib.sha256()
    for f in kernel_source_files():
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def profile_tag_order(path: str):
    """Sort key of a profiles/ file by its run tag: r01 < r01j < r01z < r01aa < r02 < r10 (numeric round, then the
    letter suffix a..z, aa..az, ...: shorter suffixes first)."""
    import re

    m = re.match(r"r(\d+)([a-z]*)_", os.path.basename(path))
    return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, "")


def pmc_traffic(kernel: str):
    """HBM bytes per launch of ``kernel`` from the newest committed rocprofv3 FETCH_SIZE summary
    (profiles/rNN[x]_pmc_fetch.csv, written by tools/profile.sh + tools/rocpd_summary.py): FETCH_SIZE is
    in KB and counts half the bytes of 16-B/lane streaming reads on gfx950 (MI355X_MICROARCH.md
    section HBM), hence x 1024 x 2.  Only a pass over THIS tree's kernels counts: its
    ``.meta.json`` must carry the current kernel_source_hash(); otherwise traffic is None and the returned
    note says why.  Returns (bytes or None, note)."""
    import csv
    import glob
    import re

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_fetch.csv")), key=profile_tag_order)
    if not files:
        return None, "no PMC pass committed"
    newest = files[-1]
    rel = os.path.relpath(newest, ROOT)
    meta = newest[: -len(".csv")] + ".meta.json"
    try:
        with open(meta) as f:
            src = json.load(f).get("kernel_source_sha256")
    except (OSError, ValueError):
        src = None
    if src != kernel_source_hash():
        return None, f"{rel} measured other kernel sources (stale, not reported)"
    with open(newest) as f:
        for row in csv.DictReader(f):
            if row["Counter"] == "FETCH_SIZE" and kernel in row["Name"]:
                return float(row["Mean"]) * 1024 * 2, rel + " (FETCH_SIZE KB x1024 x2, same kernel sources)"
    return None, f"{rel} has no {kernel} row"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--max-length", type=int, default=128)
    ap.add_argument("--model", default="large-v3")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-batch", type=int, default=4)
    ap.add_argument("--cpu-threads", type=int, default=None)
    ap.add_argument("--kernel-iters", type=int, default=20)
    ap.add_argument("--inflight", default="",
                    help="extra measurements (not the headline value), e.g. '2,3': how many bs-32 batches decode at "
                         "once, one host thread and stream each over engine lanes sharing the weights.  Off by default, "
                         "so that the rocprofv3 trace of the default command times the kernels one batch at a time, as "
                         "the roofline's live measurement does (profiles/r04k_bench.json holds a run with '2,3')")
    ap.add_argument("--stub", action="store_true",
                    help="no GPU work: each rank times a trivial host step (tests the launcher, barriers, "
                         "max-over-ranks timing and the ids gather on the CPU; with KW_BENCH_BACKEND=gloo)")
    return ap.parse_args(argv)


def launch_ranks(a, argv) -> int:
    """``--gpus N`` (N > 1) without WORLD_SIZE: one process per GPU under torch.distributed.run, started as a
    child (never exec: this process has not touched the GPU and stays the parent), rank 0's JSON line
    relayed.  Returns the launcher's exit code."""
    import socket
    import subprocess

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "16")
    proc = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, text=True)
    line = None
    for ln in proc.stdout.splitlines():
        if ln.startswith("{") and '"metric"' in ln:
            line = ln
        else:
            print(ln, flush=True)
    if line is not None:
        print(line, flush=True)
    return proc.returncode if line is not None or proc.returncode else 1


def stub_main(a, world, rank, dist):
    """The multi-rank bench skeleton without a GPU: a fixed host step per rank, the same barrier +
    max-over-ranks timing and the same (padded) ids gather as main()."""
    import torch

    def step():
        x = torch.ones(256, 256)
        for _ in range(4):
            x = x @ x / 256.0
        return torch.full((a.batch, 8), rank, dtype=torch.int32)

    for _ in range(a.warmup):
        step()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    ids = [step() for _ in range(a.steps)]
    if dist is not None:  # the ids gather is part of the timed step
        gathered = [torch.empty_like(ids[-1]) for _ in range(world)]
        dist.all_gather(gathered, ids[-1])
        assert [int(g[0, 0]) for g in gathered] == list(range(world))
        dist.barrier()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if dist is not None:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    out = {"metric": "audio-seconds/sec (RTF) whisper-large-v3 30s@bs32", "value": world * a.batch * 30.0 * a.steps / dt,
           "unit": "audio-s/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
           "ms_per_step": dt / a.steps * 1e3, "stub": True,
           "dist": {"world": world, "backend": dist.get_backend() if dist is not None else None}}
    if rank == 0:
        print(json.dumps(out), flush=True)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    a = parse(argv)
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(launch_ranks(a, argv))  # before anything touches the GPU
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("KW_BENCH_BACKEND", "nccl")
    # under a launcher (torch.distributed.run sets WORLD_SIZE) the rank code always runs the distributed path --
    # process group, barriers, max-over-ranks timing, ids gather -- world size 1 included (tests/test_gpu_dist.py
    # runs it that way over RCCL); a plain `python bench.py` is the single-process N = 1 run
    use_dist = "WORLD_SIZE" in os.environ
    if a.stub:
        if use_dist:
            dist.init_process_group(backend)
        stub_main(a, world, rank, dist if use_dist else None)
        if use_dist:
            dist.destroy_process_group()
        return
    # one process per GPU; more ranks than GPUs only in a rehearsal (KW_BENCH_BACKEND=gloo on a 1-GPU box)
    ndev = torch.cuda.device_count()
    if ndev == 0:
        raise RuntimeError("bench.py needs a HIP device (use --stub to exercise the launcher on the CPU)")
    local = local % ndev
    if use_dist:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from kwhisper.config import PRESETS
    from kwhisper.feature_extraction import WhisperFeatureExtractor
    from kwhisper.generation import KWhisperForConditionalGeneration
    from kwhisper.synthetic import dummy_audio, synthetic_state_dict
    from kwhisper import _lib as L
    from kwhisper import ops

    shape = PRESETS[a.model]
    # the numpy recipe, seed 0: the random model tests/golden/large_v3_b32_fp32.npz pins (transformers fp32 on these
    # same 32 noise clips), so the bench decodes a trajectory the GPU tests check (test_gpu_workloads, config 3)
    sd = synthetic_state_dict(shape, 0)
    model = KWhisperForConditionalGeneration.from_state_dict(shape, sd, dtype=torch.bfloat16, device=dev)
    del sd
    torch.cuda.empty_cache()
    fe = WhisperFeatureExtractor(feature_size=shape.num_mel_bins, device=dev)
    B = a.batch
    audio = torch.from_numpy(np.stack([dummy_audio(rank * 100003 + i) for i in range(B)])).to(dev)

    gen_kw = dict(language="ja", task="transcribe", max_length=a.max_length, return_timestamps=False)
    out_ids = []

    def batches(n):
        for _ in range(n):
            yield model.generate(fe.extract(audio), **gen_kw)

    def gather_ids(mats):
        """DP gather of the timed batches' token matrices (the reference's pad_across_processes +
        gather_for_metrics, C4/C5, done once for the rank's batches): width all_reduce(MAX), rows all_gather."""
        ids = torch.stack(mats).to(torch.int32)
        L = torch.tensor([ids.shape[-1]], device=dev)
        dist.all_reduce(L, op=dist.ReduceOp.MAX)
        # padded with the tokenizer's pad id, <|endoftext|> (run_pseudo_labelling.py:339)
        pad = torch.full((*ids.shape[:-1], int(L.item())), model.generation_config.eos_token_id, dtype=torch.int32,
                         device=dev)
        pad[..., : ids.shape[-1]] = ids
        gathered = [torch.empty_like(pad) for _ in range(world)]
        dist.all_gather(gathered, pad)
        return gathered

    for ids in batches(a.warmup):
        out_ids.append(ids)
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for ids in batches(a.steps):
        out_ids.append(ids)
    gathered = gather_ids(out_ids[-a.steps:]) if use_dist else None  # inside the timed region
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], device=dev, dtype=torch.float64)
    if use_dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    new_tokens = int(out_ids[-1].shape[1])
    if gathered is not None:
        assert len(gathered) == world and all(g.shape == gathered[0].shape for g in gathered)

    def inflight_rate(n_lanes, n_batches):
        """``n_lanes`` batches of B clips in flight at once (one thread, stream, model handle and decode session
        each; the weights shared through WhisperEngine.lane()): one batch's latency-bound decode chain runs beside
        another's HBM-bound cross-attention stream (tools/lab/dual_decode.py).  Every lane is warmed up (graphs
        captured) before any thread starts, so no capture overlaps another thread's launches."""
        import threading

        lanes = [KWhisperForConditionalGeneration(model.engine.lane()) for _ in range(n_lanes)]
        streams = [L.new_stream(dev) for _ in lanes]  # HIP streams of their own (kwhisper._lib.new_stream)
        ref = out_ids[-1].cpu()
        for m, st in zip(lanes, streams):
            with torch.cuda.stream(st):
                got = m.generate(fe.extract(audio), **gen_kw)
            st.synchronize()
            assert torch.equal(got.cpu(), ref), "a lane's tokens differ from the sequential run's"
        torch.cuda.synchronize()
        errs = []

        def work(m, st, k):
            try:
                with torch.cuda.stream(st):
                    for _ in range(k):
                        m.generate(fe.extract(audio), **gen_kw)
                st.synchronize()
            except BaseException as e:  # surfaced below
                errs.append(e)

        per = [n_batches // n_lanes + (1 if i < n_batches % n_lanes else 0) for i in range(n_lanes)]
        threads = [threading.Thread(target=work, args=(m, st, k)) for m, st, k in zip(lanes, streams, per)]
        t0 = time.perf_counter()
        for th in threads:
            th.start()
        for th in threads:
            th.join()
        torch.cuda.synchronize()
        dt_ = time.perf_counter() - t0
        if errs:
            raise errs[0]
        return {"lanes": n_lanes, "batches": n_batches, "value": n_batches * B * 30.0 / dt_,
                "ms_per_batch": dt_ / n_batches * 1e3,
                "note": "NOT the headline value: batches of 32 decoded concurrently, each generate() call at bs 32"}

    lanes_list = [int(x) for x in str(a.inflight).split(",") if x.strip() and int(x) > 1]
    inflight = [inflight_rate(n, max(2 * n, a.steps)) for n in lanes_list] if lanes_list and world == 1 else None

    # ---- per-kernel measurements (HIP events on the launching stream, after the timed region) ----
    eng = model.engine
    sess = model._sessions.get((B, 1)) or model._sessions[(B, 1, 1)]
    stream = torch.cuda.current_stream(dev)
    iters = a.kernel_iters

    def time_fn(fn, n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn()
        e0.record(stream)
        for _ in range(n):
            fn()
        e1.record(stream)
        e1.synchronize()
        return e0.elapsed_time(e1) / n * 1e-3

    H, S, hd = eng.H, shape.max_source_positions, 64
    n_dec = shape.decoder_layers

    def step_kernel_times(passes=3):
        """Per-kernel device time inside the decode step: the step's launch sequence run eagerly with HIP
        events around every launch (on the launch stream), so each kernel sees the cache state the graph
        replay gives it (the other kernels' weight streams between two cross-attention launches)."""
        seq = sess._step_plans(1, fused=sess.fused_last)
        tot, cnt = {}, {}
        for _ in range(passes):
            evs = []
            for item in seq:
                tag = item[0] if isinstance(item, tuple) else getattr(item, "tag", None) or "linear"
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                sess._run([item])
                e1.record(stream)
                evs.append((tag, e0, e1))
            evs[-1][2].synchronize()
            for tag, e0, e1 in evs:
                tot[tag] = tot.get(tag, 0.0) + e0.elapsed_time(e1) * 1e3
                cnt[tag] = cnt.get(tag, 0) + 1
        return {k: round(tot[k] / cnt[k], 2) for k in tot}

    kern_us = step_kernel_times()
    qx = sess._buffers(1)["qx"]
    attn_out = sess._buffers(1)["attn"]
    ws = sess._buffers(1)["ws"]
    xc_plans = [it for it in sess._step_plans(1, fused=sess.fused_last) if getattr(it, "tag", None) == "xq_cross"]
    if xc_plans:  # the step's cross-attention is the fused query projection + K/V stream (kw_dec_xq_cross)
        def cross_all_layers():  # one launch per layer, each on its own K/V: no Infinity-Cache reuse
            for pl in xc_plans:
                pl()

        d_model = shape.d_model
        # K + V of one layer (bf16) + the query projection's weights and activation rows, per launch
        cross_bytes = 2 * B * H * S * hd * 2 + d_model * d_model * 2 + B * d_model * 2
        if ops.cross_attn_pair_kernel(B * H, S, fused=True):
            cross_kernel = "cross_attn_row_kernel<true"
            cross_note = ("cross_attn_row_kernel<true, 6> (kw_dec_xq_cross: the LayerNorm-fused query projection's "
                          "workgroups, then one workgroup per (row, head) pair streaming its six K/V chunks with the "
                          "next in flight; one launch per layer; rocprof name)")
        else:
            cross_kernel = "xq_cross_kernel"
            cross_note = ("xq_cross_kernel (kw_dec_xq_cross: LayerNorm-fused query projection + one workgroup per "
                          "(row, head, chunk), K by LDS-DMA; one launch per layer; rocprof name)")
    else:
        def cross_all_layers():  # one launch per layer, each on its own K/V: no Infinity-Cache reuse
            for li in range(n_dec):
                ops.cross_attn_step(qx, B, 1, H, hd, sess.cross[2 * li], sess.cross[2 * li + 1], S, attn_out, ws)

        cross_kernel = "cross_attn_dma_kernel"
        cross_bytes = 2 * B * H * S * hd * 2  # K + V of one layer, bf16 (algorithmic)
        cross_note = ("cross_attn_dma_kernel (decoder cross-attention K/V stream, K by LDS-DMA, one launch per "
                      "layer; rocprof name)")
    cross_t = time_fn(cross_all_layers, max(1, iters // 4)) / n_dec
    feats = fe.extract(audio)
    enc_t = time_fn(lambda: eng.encode(feats), 3)
    step_graph = sess._graph
    step_t = time_fn(lambda: step_graph.replay(), iters) if step_graph is not None else None
    ms_per_step = dt / a.steps * 1e3

    result = {
        "metric": "audio-seconds/sec (RTF) whisper-large-v3 30s@bs32",
        "value": world * B * 30.0 * a.steps / dt,
        "unit": "audio-s/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic (run_speed_eval.py noise audio, random-init large-v3 weights: kwhisper.synthetic numpy recipe seed 0, the config-3 fixture's model)",
        "config": {"workload": "config 3: whisper-large-v3 greedy generate, 30 s clips, log-mel on GPU",
                   "model": shape.name, "global_batch": B * world, "per_gpu_batch": B,
                   "max_length": a.max_length, "new_tokens": new_tokens, "seq_len": 1500,
                   "parallelism": f"dp{world}"},
        "dist": {"world": world, "rank_device": local, "device_name": torch.cuda.get_device_name(dev),
                 "backend": dist.get_backend() if use_dist else None,
                 "ids_gather": "all_gather of the padded int32 token matrices, inside the timed region"
                 if use_dist else None},
        "roofline": {"kernel": cross_note,
                     "bound": "hbm", "achieved": cross_bytes / cross_t / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": cross_bytes / cross_t / 1e9 / HBM_PEAK_GBS, "traffic": None,
                     "bytes_per_launch": cross_bytes, "avg_launch_us": cross_t * 1e6},
        "encoder_mfma": {"ms": enc_t * 1e3, "tflops": ENC_FLOP_PER_CLIP * B / enc_t / 1e12,
                         "frac": ENC_FLOP_PER_CLIP * B / enc_t / 1e12 / BF16_PEAK_TFLOPS},
        "decode_step_ms": step_t * 1e3 if step_t else None,
        "inflight": inflight,
        "decode_kernel_us": kern_us,
        "decode_kernel_us_note": ("eager launches in step order with HIP events around each: includes the host "
                                  "dispatch gap a graph replay does not have; device times per kernel are the "
                                  "rocprofv3 trace averages under profiles/"),
    }
    traffic, src = pmc_traffic(cross_kernel)
    result["roofline"]["traffic"] = traffic
    result["roofline"]["traffic_source"] = src
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        from oracle.cpu_baseline import hf_cpu_generate_rate

        cb = hf_cpu_generate_rate(shape, a.cpu_batch, a.max_length, threads=a.cpu_threads)
        result["cpu_baseline"] = {
            "value": cb["audio_seconds_per_second"], "unit": "audio-s/s", "cores": cb["threads"], "kind": "reference",
            "threads": cb["threads"], "nproc": cb["nproc"], "affinity_cpus": cb["affinity_cpus"],
            "sample": f"transformers 5.15.0 WhisperForConditionalGeneration.generate fp32 on CPU, torch "
                      f"{cb['threads']} intra-op threads = this process's CPU affinity ({cb['affinity_cpus']}) capped by "
                      f"OMP_NUM_THREADS ({os.environ.get('OMP_NUM_THREADS')}, the host-CPU share of one GPU; the node "
                      f"shows nproc {cb['nproc']}), a bounded sample of {a.cpu_batch} clips x 30 s (the config's 32-clip "
                      f"batch at the same thread count: profiles/r03_cpu_baseline_b32.json), "
                      f"greedy, {cb['new_tokens']} new tokens, {cb['seconds']:.1f} s; run_speed_eval.py:73-78 timing"}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if use_dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

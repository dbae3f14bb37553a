#!/usr/bin/env python
"""BASELINE.json configs 4 and 5 on the MI355X engine (measurement tool beside bench.py, which runs config 3).

config 4  run_pseudo_labelling.py teacher=whisper-large-v3 over a synthetic stand-in for the ReazonSpeech
          "tiny" shard: 1,768 clips whose durations match misc/data_statistics.json:1 (mean 4.37 s, min
          0.62 s, max 21.8 s, total 7,723 s), each zero-padded to 30 s; bs 32 per GPU, greedy,
          return_timestamps=True (the reference default, run_pseudo_labelling.py:99), max_length 128, ja.
          The data-parallel loop is kwhisper.pseudo_label (accelerate's shard plan, padded all-gather);
          log-mel on the GPU inside the timed region.  Reports audio-s/s over the REAL durations and over
          the padded 30 s.
config 5  kotoba-whisper-v2.0 layout (32 encoder / 2 decoder layers), beam 5 + timestamps, ASR pipeline
          with chunk_length_s=15 (a 30 s clip -> 3 windows), batch 64 windows.

Random-init weights of each architecture (no checkpoints offline); one JSON line per config on rank 0.
    python tools/bench_configs.py --config 4 [--n-clips 1768]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/bench_configs.py --config 4
    python tools/bench_configs.py --config 5 [--clips 64]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/bench_configs.py --config 5
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kotoba-whisper_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

SR = 16000


def reazon_tiny_durations(n: int = 1768, seed: int = 0) -> np.ndarray:
    from kwhisper.synthetic import reazon_durations

    return reazon_durations(n, seed)


def clip_audio(i: int, dur: float) -> np.ndarray:
    from kwhisper.synthetic import reazon_audio

    return reazon_audio(i, dur, SR)


def config4(a, world, rank, dev):
    from kwhisper.config import PRESETS
    from kwhisper.feature_extraction import WhisperFeatureExtractor
    from kwhisper.generation import KWhisperForConditionalGeneration
    from kwhisper.pseudo_label import pseudo_label, step_model
    from kwhisper.synthetic import synthetic_state_dict, synthetic_state_dict_torch

    shape = PRESETS["large-v3"]
    # the weights decide the seek passes (timestamps): numpy = the model every transformers fixture pins
    sd = synthetic_state_dict(shape, 0) if a.weights == "numpy" else synthetic_state_dict_torch(shape, seed=0, device=dev)
    model = KWhisperForConditionalGeneration.from_state_dict(shape, sd, dtype=torch.bfloat16, device=dev)
    del sd
    fe = WhisperFeatureExtractor(feature_size=shape.num_mel_bins, device=dev)
    durs = reazon_tiny_durations()[: a.n_clips]
    n = len(durs)
    # the clips live on the host like the reference's dataset; each batch is padded, copied and log-mel'd
    host = [clip_audio(i, float(d)) for i, d in enumerate(durs)]
    padded = np.zeros((n, 30 * SR), dtype=np.float32)
    for i, c in enumerate(host):
        padded[i, : len(c)] = c
    pinned = torch.from_numpy(padded).pin_memory()

    def features(idx):
        # a contiguous batch (every batch of the shard plan at W = 1, and each rank's at W > 1) is a pinned view:
        # one async DMA, no host-side gather -- what the reference's DataLoader(pin_memory=True) hands over
        i0 = idx[0]
        if list(idx) == list(range(i0, i0 + len(idx))):
            return fe.extract(pinned[i0:i0 + len(idx)].to(dev, non_blocking=True))
        return fe.extract(pinned[idx].pin_memory().to(dev, non_blocking=True))

    gen_kw = dict(language="ja", task="transcribe", max_length=a.max_length, return_timestamps=True)
    # warm-up on one batch (graph capture, workspaces)
    model.generate(features(list(range(min(a.batch, n)))), **gen_kw)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    stamps, passes = {}, {}  # by step (with lanes the steps complete on lane threads, out of order)

    def on_step(si, total):  # after each batch's tokens reached the host (and, gather="round", the gather)
        stamps[si] = time.perf_counter()
        passes[si] = int((step_model() or model).stats.get("passes", 0))

    t0 = time.perf_counter()
    ids, preds = pseudo_label(model, features, n, batch_size=a.batch, gen_kwargs=gen_kw, gather=a.gather,
                              pad_token_id=model.generation_config.eos_token_id,  # tokenizer pad = <|endoftext|>
                              on_step=on_step, lanes=a.lanes, schedule=a.schedule)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    assert ids == list(range(n))
    # per-batch seconds: completion-to-completion in step order (lanes overlap batches: no projection then)
    batch_s = np.diff([t0] + [stamps[si] for si in sorted(stamps)])
    return {"metric": "audio-seconds/sec pseudo-labelling (real durations)", "value": float(durs.sum()) / dt,
            "unit": "audio-s/s", "padded_30s_value": n * 30.0 / dt, "n_gpus": world, "clips": n,
            "audio_seconds": float(durs.sum()), "seconds": dt, "higher_is_better": True, "scaling": "strong",
            "dtype": "bf16", "data": "synthetic (ReazonSpeech-tiny duration statistics, noise audio, random weights)",
            "config": {"workload": "config 4: run_pseudo_labelling.py loop, whisper-large-v3, timestamps, greedy",
                       "per_gpu_batch": a.batch, "max_length": a.max_length, "parallelism": f"dp{world}",
                       "gather": a.gather, "lanes": a.lanes, "schedule": a.schedule, "weights": a.weights,
                       "tokens_per_clip_mean": float(np.mean([len(p) for p in preds]))},
            "batch_seconds": [round(float(x), 5) for x in batch_s], "batch_seek_passes": [passes[si] for si in sorted(passes)],
            "dp_projection": (dp_projection(batch_s, passes=[passes[si] for si in sorted(passes)])
                              if world == 1 and a.lanes == 1 else None)}


def pass_unit_makespan(batch_s, passes, W):
    """List scheduling over seek-PASS work units: a batch's first pass is a unit claimed in plan
    order; each later pass of a multi-pass batch becomes a unit of its own once the previous pass has finished (rows
    are independent -- a row's pass-k decode depends on the row, its seek and k alone: TF generation_whisper.py:785-903,
    the max_length growth :1932-1940 is a function of the pass index; the engine is batch-invariant), claimed ahead of
    fresh batches by the first idle rank.  One-pass batches cost their time; a p-pass batch of time T costs t1 (the
    one-pass median) for pass 1 and (T - t1) / (p - 1) per later pass.  Returns the makespan."""
    import heapq

    t = np.asarray(batch_s, dtype=np.float64)
    p = np.asarray(passes, dtype=np.int64)
    t1 = float(np.median(t[p == 1])) if (p == 1).any() else float(t.min())
    free = [0.0] * W
    pending = []  # (ready time, cost, batch, pass index)
    nxt, end = 0, 0.0
    while nxt < len(t) or pending:
        tf = heapq.heappop(free)
        ready = [u for u in pending if u[0] <= tf]
        if ready or nxt >= len(t):
            u = min(ready or pending)
            pending.remove(u)
            fin = max(tf, u[0]) + u[1]
            if u[3] + 1 < p[u[2]]:
                pending.append((fin, u[1], u[2], u[3] + 1))
        else:
            b, nxt = nxt, nxt + 1
            fin = tf + (t1 if p[b] > 1 else t[b])
            if p[b] > 1:
                pending.append((fin, (t[b] - t1) / (p[b] - 1), b, 1))
        heapq.heappush(free, fin)
        end = max(end, fin)
    return end


def dp_projection(batch_s, worlds=(2, 4, 8), passes=None):
    """Projected data-parallel efficiency at W ranks from W = 1 per-batch times.
    Global batch i runs on rank i % W (accelerate's shard plan; the wrapped duplicates of the last round are real
    work).  Lock step (the reference's per-batch gather, gather="round"): every round waits for its slowest batch,
    efficiency = sum over rounds of the mean batch time / sum of the max.  Deferred (gather="end", schedule static):
    ranks run free until one exchange, efficiency = (total / W) / the busiest rank's sum.  Dynamic (gather="end",
    schedule="dynamic"): the batches in plan order, each to the first idle rank (list scheduling), efficiency =
    (total / W) / the last rank's finish.  ``dynamic_x10``: the same, over ten copies of these batch times (a shard
    ten times the stand-in's 56 batches): at 7 batches per rank the job's tail -- the last claimed batch's seek
    passes, which no claim order known in advance can move earlier -- is a large part of each rank's share."""
    import heapq

    t = np.asarray(batch_s, dtype=np.float64)
    out = {}
    for W in worlds:
        n_rounds = -(-len(t) // W)
        tt = np.concatenate([t, t[: n_rounds * W - len(t)]]) if n_rounds * W > len(t) else t  # wrap-around
        r = tt.reshape(n_rounds, W)
        def listed(x):
            free = [0.0] * W
            for v in x:  # list scheduling: the next batch to the rank that frees first
                heapq.heapreplace(free, free[0] + v)
            return float(x.sum() / W / max(free))

        out[f"w{W}"] = {"lockstep": round(float(r.mean(1).sum() / r.max(1).sum()), 4),
                        "deferred": round(float(tt.sum() / W / r.sum(0).max()), 4),
                        "dynamic": round(listed(tt), 4), "dynamic_x10": round(listed(np.tile(t, 10)), 4)}
        if passes is not None:  # seek passes as work units (pass_unit_makespan), no wrap-around duplicates
            out[f"w{W}"]["dynamic_pass_units"] = round(float(t.sum() / W / pass_unit_makespan(t, passes, W)), 4)
    return out


def config5(a, world, rank, dev):
    from kwhisper.config import PRESETS
    from kwhisper.generation import KWhisperForConditionalGeneration
    from kwhisper.pipeline import ASRPipeline
    from kwhisper.synthetic import synthetic_state_dict_torch

    shape = PRESETS["kotoba-v2.0"]
    sd = synthetic_state_dict_torch(shape, seed=0, device=dev)
    model = KWhisperForConditionalGeneration.from_state_dict(shape, sd, dtype=torch.bfloat16, device=dev)
    del sd
    # W > 1: the pipeline's window batches go round-robin over the ranks (ASRPipeline.data_parallel), one
    # gather of the token matrices at the end; every rank merges the full result
    pipe = ASRPipeline(model, chunk_length_s=15, batch_size=a.batch, lanes=a.lanes, data_parallel=True,
                       generate_kwargs=dict(language="ja", task="transcribe", num_beams=5, max_length=a.max_length))
    clips = [{"array": clip_audio(i, 30.0), "sampling_rate": SR} for i in range(a.clips)]
    # warm-up (graph capture on every lane), no collective: one window batch per lane (3 windows per 30 s clip)
    pipe.data_parallel = False
    pipe(clips[: max(1, -(-a.batch * a.lanes // 3))], return_timestamps=True)  # >= one full batch per lane
    pipe.data_parallel = True
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    out = pipe(clips, return_timestamps=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return {"metric": "audio-seconds/sec ASR pipeline (chunk 15 s, beam 5, timestamps)",
            "value": a.clips * 30.0 / dt, "unit": "audio-s/s", "n_gpus": world, "clips": a.clips, "seconds": dt,
            "higher_is_better": True, "dtype": "bf16", "scaling": "strong",
            "data": "synthetic (run_speed_eval.py noise audio, random-init kotoba-whisper-v2.0 layout)",
            "config": {"workload": "config 5: kotoba-v2.0 (32 enc / 2 dec), beam 5 + timestamps, chunk_length_s 15",
                       "batch_windows": a.batch, "max_length": a.max_length, "parallelism": f"dp{world}",
                       "lanes": a.lanes,
                       "tokens_per_clip_mean": float(np.mean([len(o["tokens"]) for o in out]))}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, choices=(4, 5), required=True)
    ap.add_argument("--n-clips", type=int, default=1768)
    ap.add_argument("--clips", type=int, default=64)
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--max-length", type=int, default=128)
    ap.add_argument("--gather", choices=("round", "end"), default="end",
                    help="config 4: the reference's per-batch gather (round) or one exchange at the end")
    ap.add_argument("--weights", choices=("numpy", "torch"), default="numpy",
                    help="config 4: numpy = kwhisper.synthetic.synthetic_state_dict, the random model of the transformers "
                    "fixtures (tests pin its seek passes); torch = the device generator's (another random model)")
    ap.add_argument("--schedule", choices=("static", "dynamic"), default="dynamic",
                    help="config 4 with --gather end: accelerate's batch-to-rank plan, or each batch to the first idle "
                    "rank (pseudo_label schedule='dynamic'; the same outputs)")
    ap.add_argument("--lanes", type=int, default=1,
                    help="batches of --batch in flight per GPU (config 4: pseudo_label lanes, needs --gather end; "
                    "config 5: ASRPipeline lanes)")
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    if a.config == 4:
        a.batch = a.batch or 32
        res = config4(a, world, rank, dev)
    else:
        a.batch = a.batch or 64
        res = config5(a, world, rank, dev)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

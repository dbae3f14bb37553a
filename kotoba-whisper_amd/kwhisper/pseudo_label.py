"""Data-parallel pseudo-labelling loop: the caller side of the hot path.

Restates kotoba-whisper's ``run_pseudo_labelling.py:333-354`` without accelerate. One process per GPU;
rank r takes global batches r, r+W, r+2W, ... of the dataset (accelerate's ``BatchSamplerShard`` with
``even_batches=True``, ``split_batches=False``, ``drop_last=False``: the last round is completed by
wrapping around to the start of the dataset), each batch runs through ``model.generate``, the token
matrices are padded to a common width across ranks (``Accelerator.pad_across_processes``) and
all-gathered (``Accelerator.gather_for_metrics``: the wrapped duplicates of the final round are
dropped).  The only collectives are the per-batch width ``all_reduce(MAX)`` and the ``all_gather`` of
int64 ids (~1 KB/clip), over RCCL (``nccl``) on the GPU box or ``gloo`` on the CPU.

The gathered predictions come back in dataset order, identical to a single-process run.

Resume (SURVEY.md §5 checkpoint / resume: "skip shards whose output exists"): with ``checkpoint_dir`` every
gathered round is written there by rank 0 as ``round_<step>.npz`` (numpy, no pickle; written to a temporary
name and renamed, so a crash leaves whole files only).  A restarted run decodes only the rounds without a
file -- rank 0's view of the directory is broadcast so every rank skips the same rounds and the
collectives stay matched -- and reads the others back (one node: the directory is visible to every rank).
"""
from __future__ import annotations

import csv
import os
import threading
from typing import Callable, Iterable, List, Optional, Sequence

import numpy as np
import torch

from . import _lib

__all__ = ["shard_batches", "gather_remainder", "pad_across_processes", "gather_matrices", "pseudo_label",
           "pseudo_label_multitask", "last_schedule",
           "legacy_prompt", "write_transcription_csv", "transcription_table", "write_transcription_arrow"]


def shard_batches(n_items: int, batch_size: int, world: int, rank: int) -> List[List[int]]:
    """Dataset indices of every batch rank ``rank`` processes, in step order.

    Restates ``accelerate.data_loader.BatchSamplerShard._iter_with_no_split`` (accelerate 1.x) over a
    sequential ``BatchSampler(range(n_items), batch_size, drop_last=False)``, even_batches=True: batch
    i goes to rank i % world; a round is yielded only once every rank has a full batch, and the final
    round is completed with indices taken cyclically from the start of the dataset."""
    if n_items <= 0:
        return []
    if batch_size <= 0 or world <= 0 or not 0 <= rank < world:
        raise ValueError("batch_size and world must be positive and 0 <= rank < world")
    batches = [list(range(s, min(s + batch_size, n_items))) for s in range(0, n_items, batch_size)]
    out: List[List[int]] = []
    initial: List[int] = []
    to_yield = None
    idx = -1
    batch: List[int] = []
    for idx, batch in enumerate(batches):
        if idx < world:
            initial += batch
        if idx % world == rank:
            to_yield = batch
        if idx % world == world - 1 and len(batch) == batch_size:
            out.append(to_yield)
            to_yield = None
    if to_yield is not None and len(to_yield) == batch_size:
        out.append(to_yield)
    while len(initial) < world * batch_size:
        initial = initial + initial
    if len(batch) == batch_size:
        batch = []
        idx += 1
    cyc = 0
    while idx % world != 0 or len(batch) > 0:
        end = cyc + batch_size - len(batch)
        batch = batch + initial[cyc:end]
        if idx % world == rank:
            out.append(batch)
        cyc = end
        batch = []
        idx += 1
    return out


def gather_remainder(n_items: int, batch_size: int, world: int) -> int:
    """Items of the final gathered round that are real (``GradientState.remainder``); 0 = all."""
    return n_items % (batch_size * world)


def _dist():
    import torch.distributed as dist

    return dist if dist.is_available() and dist.is_initialized() else None


def pad_across_processes(ids: torch.Tensor, pad_index: int) -> torch.Tensor:
    """Right-pad dim 1 to the widest rank's (``Accelerator.pad_across_processes(dim=1)``).  Whenever a process
    group is initialised the collective runs, world size 1 included (so a one-rank RCCL run exercises it)."""
    dist = _dist()
    if dist is None:
        return ids
    w = torch.tensor([ids.shape[1]], dtype=torch.int64, device=ids.device)
    dist.all_reduce(w, op=dist.ReduceOp.MAX)
    T = int(w.item())
    if T == ids.shape[1]:
        return ids
    out = torch.full((ids.shape[0], T), pad_index, dtype=ids.dtype, device=ids.device)
    out[:, : ids.shape[1]] = ids
    return out


def _all_gather_rows(t: torch.Tensor) -> torch.Tensor:
    dist = _dist()
    if dist is None:
        return t
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t.contiguous())
    return torch.cat(parts, 0)


def legacy_prompt(generation_config, language: str, task: str = "transcribe", return_timestamps: bool = False):
    """The init tokens older transformers (4.35, the reference's pin ``requirements.txt:2``) left at the start
    of every generated row: ``[sot, lang, task]`` plus ``notimestamps`` without timestamps
    (generation_whisper.py:1591-1603).  The legacy consumer ``run_data_filtering.py:230-251,279`` reads the
    task tokens at ``timestamp_position = 3`` of each row."""
    from .config import language_to_id

    g = generation_config
    row = [g.decoder_start_token_id, language_to_id(language, g), g.task_to_id[task]]
    if not return_timestamps:
        row.append(g.no_timestamps_token_id)
    return row


def _with_prompt(ids: torch.Tensor, prompt: Sequence[int]) -> torch.Tensor:
    pre = torch.tensor(list(prompt), dtype=ids.dtype, device=ids.device).expand(ids.shape[0], len(prompt))
    return torch.cat([pre, ids], 1)


def _round_path(checkpoint_dir: str, si: int) -> str:
    return os.path.join(checkpoint_dir, f"round_{si:06d}.npz")


def _rank_round_path(checkpoint_dir: str, si: int, rank: int) -> str:
    return os.path.join(checkpoint_dir, f"round_{si:06d}_rank{rank:03d}.npz")


def _batch_path(checkpoint_dir: str, j: int) -> str:
    return os.path.join(checkpoint_dir, f"batch_{j:06d}.npz")


def weights_fingerprint(model) -> Optional[str]:
    """A short digest of a few of the model's weight values (the token embedding's first rows and the decoder's
    last layer's fc2 bias), so a resume with other weights of the same architecture is refused; None for a
    model without an engine (test stubs)."""
    import hashlib

    eng = getattr(model, "engine", None)
    if eng is None or getattr(eng, "tok_emb", None) is None:
        return None
    parts = [eng.tok_emb[:8].float().cpu().numpy().tobytes()]
    lay = (getattr(eng, "dec_layers", None) or [None])[-1]
    if isinstance(lay, dict) and lay.get("fc2_b") is not None:
        parts.append(lay["fc2_b"].float().cpu().numpy().tobytes())
    return hashlib.sha256(b"".join(parts)).hexdigest()[:16]


def run_digest(model, **config) -> str:
    """A stable digest of what decides the labels besides the item plan: the generate kwargs, the output
    layout options and the model (its architecture name, compute dtype and a fingerprint of its weights).  A
    resume with any of them changed would mix two configurations' rounds, so ``plan.json`` records it (sha256
    of sorted JSON)."""
    import hashlib
    import json

    shape = getattr(getattr(model, "config", None), "shape", None)
    ident = {"model": getattr(shape, "name", None) or type(model).__name__, "dtype": str(getattr(model, "dtype", ""))}
    fp = weights_fingerprint(model)
    if fp is not None:
        ident["weights"] = fp
    blob = json.dumps({"model": ident, **config}, sort_keys=True, default=repr)
    return hashlib.sha256(blob.encode()).hexdigest()


def _plan_matches(stored: dict, plan: dict, allow_legacy: bool = False) -> bool:
    """plan.json equality.  A plan written before the configuration digest existed (no ``config_sha256``) cannot
    prove that its rounds were decoded with this run's generate kwargs and weights, so it is refused unless the
    caller opts in (``allow_legacy_checkpoint=True``), and then resumed with a warning."""
    if stored == plan:
        return True
    legacy = "config_sha256" not in stored and {k: v for k, v in plan.items() if k != "config_sha256"} == stored
    if legacy and allow_legacy:
        import warnings

        warnings.warn("checkpoint plan.json predates the configuration digest: resuming without checking that the "
                      "generate kwargs / model match the rounds on disk", RuntimeWarning, stacklevel=3)
        return True
    return False


def _done_rounds(checkpoint_dir: Optional[str], n_steps: int, device, plan: dict, rank_files: int = 0,
                 batch_files: bool = False, allow_legacy: bool = False) -> List[bool]:
    """Which gathered rounds already have a checkpoint file, as rank 0 sees it (broadcast: every rank skips
    the same rounds, so the per-round collectives stay matched).  The directory's ``plan.json`` (items,
    batch size, world size, and the digest of the generate kwargs / output layout / model) must match this
    run's: the rounds of another plan hold other items or other labels.  ``rank_files`` = W (deferred gather):
    a round counts as done when every rank's own file of it exists.  ``batch_files`` (dynamic schedule): entry j is
    global batch j's ``batch_<j>.npz``."""
    if not checkpoint_dir or n_steps == 0:
        return [False] * n_steps
    import json

    dist = _dist()
    rank = dist.get_rank() if dist else 0
    mask = torch.zeros((n_steps + 1,), dtype=torch.int64, device=device)  # [0]: 1 = plan mismatch
    if rank == 0:
        meta = os.path.join(checkpoint_dir, "plan.json")
        if os.path.exists(meta):
            with open(meta) as f:
                mask[0] = int(not _plan_matches(json.load(f), plan, allow_legacy))
        else:
            with open(meta + ".tmp", "w") as f:
                json.dump(plan, f)
            os.replace(meta + ".tmp", meta)
        if not int(mask[0]):
            for si in range(n_steps):
                if batch_files:
                    ok = os.path.exists(_batch_path(checkpoint_dir, si))
                elif rank_files:
                    ok = all(os.path.exists(_rank_round_path(checkpoint_dir, si, r)) for r in range(rank_files))
                else:
                    ok = os.path.exists(_round_path(checkpoint_dir, si))
                mask[si + 1] = int(ok)
    if dist is not None and dist.get_world_size() > 1:
        dist.broadcast(mask, 0)
    m = mask.cpu().tolist()
    if m[0]:
        raise ValueError(f"checkpoint_dir {checkpoint_dir} holds rounds of another plan than {plan} (plan.json; a plan "
                         "without config_sha256 predates the digest: pass allow_legacy_checkpoint=True to resume it)")
    return [bool(x) for x in m[1:]]


def _save_round(checkpoint_dir: str, si: int, fid: List[int], mats: List[np.ndarray], path: Optional[str] = None,
                rank: Optional[int] = None) -> None:
    path = path or _round_path(checkpoint_dir, si)
    tmp = f"{path}.{os.getpid()}.{threading.get_ident()}.tmp"
    extra = {} if rank is None else {"rank": np.asarray(rank, dtype=np.int64)}  # dynamic schedule: who decoded it
    with open(tmp, "wb") as f:
        np.savez(f, fid=np.asarray(fid, dtype=np.int64), **extra, **{f"c{c}": m for c, m in enumerate(mats)})
    os.replace(tmp, path)  # atomic: a restart sees the whole round or none of it


def _load_round(checkpoint_dir: str, si: int, path: Optional[str] = None):
    with np.load(path or _round_path(checkpoint_dir, si), allow_pickle=False) as z:
        n_cols = sum(1 for k in z.files if k.startswith("c") and k[1:].isdigit())
        return z["fid"].tolist(), [z[f"c{c}"] for c in range(n_cols)]


def _label_loop(model, features, n_items, batch_size, pad_token_id, comm_device, on_step, decode,
                checkpoint_dir=None, digest=None, schedule="static", allow_legacy=False):
    """Shared DP loop: ``decode(feats)`` -> list of id matrices (one per output column); each is padded
    across ranks and gathered with the file ids (``run_pseudo_labelling.py:336-344``, v3 ``:309-321``).
    With ``checkpoint_dir``, gathered rounds are checkpointed and rounds already on disk are skipped."""
    if schedule != "static":
        raise ValueError("schedule='dynamic' needs gather='end' (the per-round gather keeps the ranks in lock step)")
    dist = _dist()
    world = dist.get_world_size() if dist else 1
    rank = dist.get_rank() if dist else 0
    steps = shard_batches(n_items, batch_size, world, rank)
    rem = gather_remainder(n_items, batch_size, world)
    if checkpoint_dir and rank == 0:
        os.makedirs(checkpoint_dir, exist_ok=True)
    mask_dev = comm_device if comm_device is not None else (
        torch.device("cuda", torch.cuda.current_device()) if dist is not None and dist.get_backend() == "nccl"
        else torch.device("cpu"))
    done = _done_rounds(checkpoint_dir, len(steps), mask_dev,
                        {"n_items": int(n_items), "batch_size": int(batch_size), "world_size": int(world),
                         "config_sha256": digest}, allow_legacy=allow_legacy)
    eval_ids: List[int] = []
    cols: Optional[List[List[np.ndarray]]] = None
    for si, idx in enumerate(steps):
        if done[si]:  # decoded by an earlier run: read the gathered round back
            fid_l, mats = _load_round(checkpoint_dir, si)
            if cols is None:
                cols = [[] for _ in mats]
            if len(mats) != len(cols):
                raise ValueError(f"checkpoint {_round_path(checkpoint_dir, si)} holds {len(mats)} output columns, "
                                 f"this run produces {len(cols)}")
            eval_ids.extend(fid_l)
            for c, m in enumerate(mats):
                cols[c].extend(m)
            if on_step is not None:
                on_step(si, len(steps))
            continue
        outs = decode(features(idx))
        if cols is None:
            cols = [[] for _ in outs]
        last = si == len(steps) - 1 and rem > 0
        fid = None
        round_fid: List[int] = []
        round_mats: List[np.ndarray] = []
        for c, ids in enumerate(outs):
            ids = ids.to(comm_device) if comm_device is not None else ids
            ids = _all_gather_rows(pad_across_processes(ids, pad_token_id))
            if fid is None:
                fid = _all_gather_rows(torch.tensor(idx, dtype=torch.int64, device=ids.device))
                if last:
                    fid = fid[:rem]
                round_fid = [int(x) for x in fid.cpu().tolist()]
                eval_ids.extend(round_fid)
            if last:
                ids = ids[:rem]
            mat = ids.cpu().numpy()
            round_mats.append(mat)
            cols[c].extend(mat)
        if checkpoint_dir and rank == 0:
            _save_round(checkpoint_dir, si, round_fid, round_mats)
        if on_step is not None:
            on_step(si, len(steps))
    return eval_ids, cols or []


class _Claims:
    """The next global batch index for a worker (a rank's lane thread): ONE counter shared by every rank, held in the
    process group's own key-value store (``Store.add`` on the rendezvous TCPStore: a host round trip, the GPU is never
    involved), so the next batch goes to the first idle worker anywhere in the job.  Without a process group: a local
    counter.  ``order`` maps the k-th claim to a global batch index (the batches not already on disk)."""

    _calls = 0  # per process; every rank makes the same sequence of pseudo_label calls, so keys match

    def __init__(self, dist, order: List[int]):
        self.order, self.lock = order, threading.Lock()
        self.store, self.key, self.local = None, None, 0
        if dist is not None:
            from torch.distributed import distributed_c10d as c10d

            _Claims._calls += 1
            self.store = c10d._get_default_store()
            self.key = f"kwhisper/pseudo_label/{_Claims._calls}/next"

    def next(self) -> Optional[int]:
        with self.lock:  # one store client per process: lane threads take turns
            if self.store is not None:
                k = int(self.store.add(self.key, 1)) - 1
            else:
                k, self.local = self.local, self.local + 1
        return self.order[k] if k < len(self.order) else None


_LAST_SCHEDULE: List[int] = []


def last_schedule() -> List[int]:
    """After a ``schedule="dynamic"`` call: the rank that decoded each global batch (round si, rank slot r ->
    index si * W + r of the reference's plan), -1 for a batch read back from ``checkpoint_dir``."""
    return list(_LAST_SCHEDULE)


def _label_loop_deferred(model, features, n_items, batch_size, pad_token_id, comm_device, on_step, decode,
                         checkpoint_dir=None, digest=None, schedule="static", allow_legacy=False):
    """``_label_loop`` with the per-round collectives deferred to ONE exchange at the end (``gather="end"``).

    The reference pads and gathers after every batch (run_pseudo_labelling.py:339-341), so every round waits
    for the slowest rank's batch; with timestamps a batch's cost depends on its seek passes, so that lock step
    loses throughput at W > 1.  Here each rank decodes its batches without a collective, keeps its per-batch
    matrices and widths, and at the end one all-reduce(MAX) of the width and two all-gathers (per-batch shapes, the
    padded token rows) rebuild exactly the rounds the per-batch gather would have produced: each round's rows padded
    to that round's widest rank, the wrapped duplicates of the final round dropped, file ids from the
    (deterministic) shard plan of every rank.

    ``schedule="static"``: rank r decodes accelerate's batches r, r + W, ... (``shard_batches``).  Resume: each rank
    checkpoints its own batches (``round_<step>_rank<r>.npz``); a round counts as done when every rank's file of it
    exists (rank 0's view, broadcast once).
    ``schedule="dynamic"``: the same W x n_steps batches (identical item sets, so identical outputs -- the decode of a
    batch does not depend on the process that runs it), but each worker (every lane of every rank) takes the NEXT
    undecoded batch when it becomes idle (``_Claims``: list scheduling), so a rank that drew a slow batch (several seek
    passes) no longer holds the others back.  Resume: one file per global batch (``batch_<j>.npz``, with the rank that
    decoded it); batches on disk are skipped and read back by every rank.  ``last_schedule()`` reports who decoded what.
    ``on_step(step, total)`` is called from the decoding thread, one call at a time (a lock), in completion order;
    ``step`` is the rank's step index (static) or the global batch index (dynamic)."""
    global _LAST_SCHEDULE
    dist = _dist()
    world = dist.get_world_size() if dist else 1
    rank = dist.get_rank() if dist else 0
    plans = [shard_batches(n_items, batch_size, world, r) for r in range(world)]
    n_steps = len(plans[rank])
    rem = gather_remainder(n_items, batch_size, world)
    if schedule not in ("static", "dynamic"):
        raise ValueError(f"schedule must be 'static' or 'dynamic', got {schedule!r}")
    dynamic = schedule == "dynamic"
    if checkpoint_dir and rank == 0:
        os.makedirs(checkpoint_dir, exist_ok=True)
    dev = comm_device if comm_device is not None else (
        torch.device("cuda", torch.cuda.current_device()) if dist is not None and dist.get_backend() == "nccl"
        else torch.device("cpu"))
    plan = {"n_items": int(n_items), "batch_size": int(batch_size), "world_size": int(world),
            "config_sha256": digest, "gather": "end"}
    n_global = n_steps * world
    if dynamic:
        plan["schedule"] = "dynamic"
        done = _done_rounds(checkpoint_dir, n_global, dev, plan, batch_files=True, allow_legacy=allow_legacy)
    else:
        done = _done_rounds(checkpoint_dir, n_steps, dev, plan, rank_files=world, allow_legacy=allow_legacy)
    decoders = decode if isinstance(decode, (list, tuple)) else [decode]
    step_lock = threading.Lock()  # on_step: one call at a time, whichever lane thread finished the batch
    # static: local[si] = the rank's step si; dynamic: mine[j] = global batch j decoded here
    local: List[Optional[List[np.ndarray]]] = [None] * n_steps
    mine: dict = {}

    def gbatch(j):  # global batch j = round j // W, rank slot j % W of the reference's plan
        return plans[j % world][j // world]

    def report(si, total):
        if on_step is not None:
            with step_lock:
                on_step(si, total)

    def run_step(si, dec):
        idx = steps[si]
        path = _rank_round_path(checkpoint_dir, si, rank) if checkpoint_dir else None
        if done[si]:
            _, mats = _load_round(checkpoint_dir, si, path)
        else:
            mats = [o.cpu().numpy().astype(np.int64) for o in dec(features(idx))]
            if checkpoint_dir:
                _save_round(checkpoint_dir, si, list(idx), mats, path)
        local[si] = mats
        report(si, n_steps)

    def run_global(j, dec):
        idx = gbatch(j)
        mats = [o.cpu().numpy().astype(np.int64) for o in dec(features(idx))]
        if checkpoint_dir:
            _save_round(checkpoint_dir, j, list(idx), mats, _batch_path(checkpoint_dir, j), rank=rank)
        mine[j] = mats
        report(j, n_global)

    steps = plans[rank]
    errs: List[BaseException] = []
    import contextlib

    # each lane on its own stream of this rank's device (on one shared stream the lanes would serialise; a new
    # thread's current device is 0, the stream context sets it)
    n = len(decoders)
    streams = [_lib.new_stream(torch.cuda.current_device()) for _ in range(n)] \
        if n > 1 and torch.cuda.is_available() else [None] * n

    def in_lane(i, work):
        try:
            ctx = torch.cuda.stream(streams[i]) if streams[i] is not None else contextlib.nullcontext()
            with ctx:
                work()
        except BaseException as e:  # re-raised on the calling thread
            errs.append(e)

    def run_threads(works):
        if len(works) == 1:
            works[0]()
            return
        threads = [threading.Thread(target=in_lane, args=(i, w)) for i, w in enumerate(works)]
        for th in threads:
            th.start()
        for th in threads:
            th.join()
        for st in streams:  # (recycled by the next call's lanes: _lib.new_stream)
            if st is not None:
                _lib.release_stream(st)
        if errs:
            raise errs[0]

    if dynamic:
        claims = _Claims(dist, [j for j in range(n_global) if not done[j]])

        def worker(dec):
            def work():
                while (j := claims.next()) is not None:
                    run_global(j, dec)
            return work

        # lanes capture their graphs on their own threads (captures serialised by decode.CAPTURE_LOCK)
        run_threads([worker(d) for d in decoders])
    elif n == 1:
        for si in range(n_steps):
            run_step(si, decoders[0])
    else:  # lanes: step si on lane si % n (one host thread each)
        def lane_steps(i):
            def work():
                for si in range(i, n_steps, n):
                    run_step(si, decoders[i])
            return work

        run_threads([lane_steps(i) for i in range(n)])

    if dynamic:  # every rank's decoded batches, by global index; batches on disk read back here
        js = sorted(mine)
        outs = [mine[j] for j in js]
    else:
        outs = local
    for k, mats in enumerate(outs):
        if len(mats) != len(outs[0]):
            raise ValueError(f"batch {k} produced {len(mats)} output columns, earlier batches {len(outs[0])}")
    n_cols = len(outs[0]) if outs else 0
    if dist is not None:  # agree on the column count (a rank may have decoded nothing)
        t = torch.tensor([n_cols], dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        n_cols = int(t.item())
    if dynamic:
        n_cols = _dynamic_columns(n_cols, done, checkpoint_dir)
        by_j: List[Optional[List[np.ndarray]]] = [None] * n_global
        owner = [-1] * n_global
        n_slots = len(js)
        if dist is not None:
            t = torch.tensor([n_slots], dtype=torch.int64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            n_slots = int(t.item())
        # the global indices travel as one more matrix per rank; each column's matrices as one gather
        idx_all = gather_matrices([np.asarray([js], dtype=np.int64).reshape(1, -1)], 1, -1, dev)
        per_col = [gather_matrices([m[c] for m in outs], n_slots, pad_token_id, dev) for c in range(n_cols)]
        for r in range(world):
            for k, j in enumerate(idx_all[r][0].reshape(-1).tolist() if idx_all[r] else []):
                by_j[j] = [per_col[c][r][k] for c in range(n_cols)]
                owner[j] = r
        for j in range(n_global):
            if done[j]:
                _, by_j[j] = _load_round(checkpoint_dir, j, _batch_path(checkpoint_dir, j))
        _LAST_SCHEDULE = owner
        per_rank_cols = [[[by_j[si * world + r][c] for si in range(n_steps)] for r in range(world)]
                         for c in range(n_cols)]
    else:
        per_rank_cols = [gather_matrices([m[c] for m in local], n_steps, pad_token_id, dev) for c in range(n_cols)]
    eval_ids: List[int] = []
    for si in range(n_steps):
        fid = [i for r in range(world) for i in plans[r][si]]
        eval_ids.extend(fid[:rem] if si == n_steps - 1 and rem > 0 else fid)
    cols: List[List[np.ndarray]] = []
    for c in range(n_cols):
        per_rank = per_rank_cols[c]
        out: List[np.ndarray] = []
        for si in range(n_steps):
            w = max(per_rank[r][si].shape[1] for r in range(world))  # the round's common width
            rnd = []
            for r in range(world):
                m = per_rank[r][si]
                pm = np.full((m.shape[0], w), pad_token_id, dtype=np.int64)
                pm[:, : m.shape[1]] = m
                rnd.append(pm)
            mat = np.concatenate(rnd, 0)
            if si == n_steps - 1 and rem > 0:
                mat = mat[:rem]
            out.extend(mat)
        cols.append(out)
    return eval_ids, cols


def _dynamic_columns(n_cols: int, done: List[bool], checkpoint_dir: Optional[str]) -> int:
    """Output columns when no rank decoded anything this run (every batch resumed from disk)."""
    if n_cols or not any(done):
        return n_cols
    j = done.index(True)
    return len(_load_round(checkpoint_dir, j, _batch_path(checkpoint_dir, j))[1])


def gather_matrices(mats: Sequence[np.ndarray], n_slots: int, pad: int, device=None) -> List[List[np.ndarray]]:
    """Every rank's list of int64 matrices, on every rank, exactly as each rank held them (shapes included): one
    all_reduce(MAX) of the largest shape, then all_gathers of the shapes and of the matrices padded to it.
    ``n_slots`` >= the longest list over ranks (unused slots travel as padding).  Without a process group: [mats]."""
    dist = _dist()
    mats = [np.asarray(m, dtype=np.int64).reshape(np.shape(m)[0], -1) for m in mats]
    if dist is None:
        return [list(mats)]
    if len(mats) > n_slots:
        raise ValueError(f"{len(mats)} matrices for {n_slots} slots")
    world = dist.get_world_size()
    dev = device if device is not None else (
        torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu"))
    big = torch.tensor([max([m.shape[0] for m in mats], default=0), max([m.shape[1] for m in mats], default=0)],
                       dtype=torch.int64, device=dev)
    dist.all_reduce(big, op=dist.ReduceOp.MAX)
    R, T = max(int(big[0]), 1), max(int(big[1]), 1)
    shapes = np.full((n_slots, 2), -1, dtype=np.int64)  # -1: unused slot
    buf = np.full((n_slots, R, T), pad, dtype=np.int64)
    for i, m in enumerate(mats):
        shapes[i] = m.shape
        buf[i, : m.shape[0], : m.shape[1]] = m
    g_s = _all_gather_rows(torch.from_numpy(shapes).to(dev)).view(world, n_slots, 2).cpu().numpy()
    g_b = _all_gather_rows(torch.from_numpy(buf).to(dev)).view(world, n_slots, R, T).cpu().numpy()
    return [[g_b[r, i, : g_s[r, i, 0], : g_s[r, i, 1]] for i in range(n_slots) if g_s[r, i, 0] >= 0]
            for r in range(world)]


_GATHER = {"round": _label_loop, "end": _label_loop_deferred}
_STEP = threading.local()


def step_model():
    """Inside an ``on_step`` callback: the model handle (the caller's model or one of its lanes) that decoded the
    step just reported -- with ``lanes`` > 1 the steps run on lane threads, each lane's ``stats`` its own."""
    return getattr(_STEP, "model", None)


def _lane_models(model, lanes: int, gather: str):
    if lanes < 1:
        raise ValueError("lanes must be >= 1")
    if lanes == 1:
        return [model]
    if gather != "end":
        raise ValueError("lanes > 1 needs gather='end' (the per-round gather keeps one batch in flight)")
    if not hasattr(model, "lane"):
        raise ValueError("lanes > 1 needs a model with lane() (an independent handle on the same weights)")
    return [model] + [model.lane() for _ in range(lanes - 1)]


def _loop(gather):
    try:
        return _GATHER[gather]
    except KeyError:
        raise ValueError(f"gather must be 'round' (the reference's per-batch gather) or 'end', got {gather!r}") from None


def pseudo_label(model, features: Callable[[Sequence[int]], torch.Tensor], n_items: int, *, batch_size: int,
                 pad_token_id: int, gen_kwargs: Optional[dict] = None, comm_device=None,
                 on_step: Optional[Callable[[int, int], None]] = None, legacy_prompt_in_output: bool = False,
                 checkpoint_dir: Optional[str] = None, gather: str = "round", lanes: int = 1,
                 schedule: str = "static", allow_legacy_checkpoint: bool = False):
    """Transcribe items 0..n_items-1 data-parallel; returns (item_indices, predictions) in dataset order
    on every rank (``run_pseudo_labelling.py:333-344``).

    ``features(indices)`` returns the (b, n_mels, 3000) log-mel batch for those dataset indices (on the
    model's device); ``predictions`` is a list of 1-D int64 numpy arrays, one per item, each padded to
    its gather round's common width exactly as the reference's ``eval_preds`` rows are.
    ``pad_token_id`` is required and is the TOKENIZER's pad id, as the reference pads across processes with
    ``tokenizer.pad_token_id`` (run_pseudo_labelling.py:339) -- for the Whisper tokenizers that is
    ``<|endoftext|>`` (the eos id, 50257), not ``generation_config.pad_token_id`` (50256), which only pads
    rows inside one generate() output.
    ``legacy_prompt_in_output`` prepends ``legacy_prompt(...)`` to every row (needs ``language``).
    ``checkpoint_dir``: checkpoint every gathered round there and skip rounds already written (resume).
    ``gather``: "round" pads and gathers after every batch as the reference does; "end" defers every collective
    to one exchange after the rank's last batch (``_label_loop_deferred``: the same predictions, no lock step).
    ``lanes`` > 1 (with gather="end"): that many of the rank's batches decode at once, each batch still
    ``batch_size`` items, on ``model.lane()`` handles (shared weights, one host thread and stream each): one
    batch's latency-bound decode chain overlaps another's HBM-bound cross-attention (tools/lab/dual_decode.py).
    ``schedule`` (with gather="end"): "static" = accelerate's batch-to-rank plan; "dynamic" = the same batches, each
    taken by the first idle worker of any rank (``_label_loop_deferred``).  The predictions are the same.
    ``on_step(step, total)`` runs on the thread that decoded the step (a lane thread with lanes > 1), one call at a
    time, in completion order.  ``allow_legacy_checkpoint``: resume a ``checkpoint_dir`` whose plan.json predates
    the configuration digest (refused by default)."""
    gen_kwargs = dict(gen_kwargs or {})
    loop = _loop(gather)
    models = _lane_models(model, lanes, gather)
    prompt = None
    if legacy_prompt_in_output:
        if not gen_kwargs.get("language"):
            raise ValueError("legacy_prompt_in_output needs an explicit `language` in gen_kwargs")
        prompt = legacy_prompt(model.generation_config, gen_kwargs["language"], gen_kwargs.get("task") or "transcribe",
                               bool(gen_kwargs.get("return_timestamps")))

    def decoder(m):
        def decode(feats):
            _STEP.model = m  # (step_model(): the lane handle whose stats an on_step callback should read)
            ids = m.generate(feats, **gen_kwargs)
            return [_with_prompt(ids, prompt) if prompt else ids]

        return decode

    digest = run_digest(model, gen_kwargs=gen_kwargs, pad_token_id=int(pad_token_id),
                        legacy_prompt_in_output=bool(legacy_prompt_in_output)) if checkpoint_dir else None
    decs = [decoder(m) for m in models]
    eval_ids, cols = loop(model, features, n_items, batch_size, pad_token_id, comm_device, on_step,
                          decs if len(decs) > 1 else decs[0], checkpoint_dir, digest, schedule=schedule,
                          allow_legacy=allow_legacy_checkpoint)
    return eval_ids, (cols[0] if cols else [])


def pseudo_label_multitask(model, features: Callable[[Sequence[int]], torch.Tensor], n_items: int, *,
                           batch_size: int, text_lang_task: Sequence[tuple], pad_token_id: int,
                           gen_kwargs: Optional[dict] = None, comm_device=None,
                           on_step: Optional[Callable[[int, int], None]] = None, checkpoint_dir: Optional[str] = None,
                           gather: str = "round", schedule: str = "static", allow_legacy_checkpoint: bool = False):
    """``run_pseudo_labelling_v3.py:299-321``: every batch is decoded once per (text, lang, task) triple.
    Returns (item_indices, {text: predictions}) in dataset order; ``whisper_<text>`` is the column the
    reference adds (:322-323).  The encoder and cross-K/V run once per batch (``generate_multitask``) when
    the model offers it, so each extra task costs only its decode loop."""
    gen_kwargs = dict(gen_kwargs or {})
    loop = _loop(gather)
    tasks = [(lang, task) for _, lang, task in text_lang_task]

    def decode(feats):
        if hasattr(model, "generate_multitask"):
            return model.generate_multitask(feats, tasks, **gen_kwargs)
        return [model.generate(feats, language=lang, task=task, **gen_kwargs) for lang, task in tasks]

    digest = run_digest(model, gen_kwargs=gen_kwargs, pad_token_id=int(pad_token_id),
                        text_lang_task=[list(t) for t in text_lang_task]) if checkpoint_dir else None
    eval_ids, cols = loop(model, features, n_items, batch_size, pad_token_id, comm_device, on_step, decode,
                          checkpoint_dir, digest, schedule=schedule, allow_legacy=allow_legacy_checkpoint)
    if not cols:
        cols = [[] for _ in text_lang_task]
    return eval_ids, {t[0]: c for t, c in zip(text_lang_task, cols)}


def write_transcription_csv(path: str, file_ids: Iterable[str], preds: Iterable[np.ndarray]) -> None:
    """``train-transcription.csv`` exactly as run_pseudo_labelling.py:347-350 writes it: a header row
    then ``[file_id, str(ndarray)]`` per item (numpy's default array repr of the token row)."""
    with open(path, "w", encoding="UTF8", newline="") as f:
        w = csv.writer(f)
        w.writerow(["file_id", "whisper_transcript"])
        w.writerows([[fid, p] for fid, p in zip(file_ids, preds)])


def transcription_table(file_ids: Iterable[str], preds: Iterable[np.ndarray], column: str = "whisper_transcript"):
    """The pseudo-label Arrow column the reference appends to the dataset
    (``raw_datasets["train"].add_column("whisper_transcript", eval_preds)``, run_pseudo_labelling.py:351):
    ``list<int64>`` token rows, keyed by ``file_id``."""
    import pyarrow as pa

    rows = [np.asarray(p, dtype=np.int64) for p in preds]
    return pa.table({"file_id": pa.array(list(file_ids), type=pa.string()),
                     column: pa.array([r.tolist() for r in rows], type=pa.list_(pa.int64()))})


def write_transcription_arrow(path: str, file_ids: Iterable[str], preds: Iterable[np.ndarray],
                              column: str = "whisper_transcript") -> None:
    """Write ``transcription_table`` as an Arrow IPC stream file (the format of ``datasets``' cache files)."""
    import pyarrow as pa

    table = transcription_table(file_ids, preds, column)
    with pa.OSFile(path, "wb") as sink, pa.ipc.new_stream(sink, table.schema) as w:
        w.write_table(table)

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
"""
from __future__ import annotations

import csv
from typing import Callable, Iterable, List, Optional, Sequence

import numpy as np
import torch

__all__ = ["shard_batches", "gather_remainder", "pad_across_processes", "pseudo_label", "write_transcription_csv"]


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
    """Right-pad dim 1 to the widest rank's (``Accelerator.pad_across_processes(dim=1)``)."""
    dist = _dist()
    if dist is None or dist.get_world_size() == 1:
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
    if dist is None or dist.get_world_size() == 1:
        return t
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t.contiguous())
    return torch.cat(parts, 0)


def pseudo_label(model, features: Callable[[Sequence[int]], torch.Tensor], n_items: int, *, batch_size: int,
                 gen_kwargs: Optional[dict] = None, pad_token_id: int = 50256, comm_device=None,
                 on_step: Optional[Callable[[int, int], None]] = None):
    """Transcribe items 0..n_items-1 data-parallel; returns (item_indices, predictions) in dataset order
    on every rank (``run_pseudo_labelling.py:333-344``).

    ``features(indices)`` returns the (b, n_mels, 3000) log-mel batch for those dataset indices (on the
    model's device); ``predictions`` is a list of 1-D int64 numpy arrays, one per item, each padded to
    its gather round's common width exactly as the reference's ``eval_preds`` rows are."""
    dist = _dist()
    world = dist.get_world_size() if dist else 1
    rank = dist.get_rank() if dist else 0
    gen_kwargs = dict(gen_kwargs or {})
    steps = shard_batches(n_items, batch_size, world, rank)
    rem = gather_remainder(n_items, batch_size, world)
    eval_ids: List[int] = []
    eval_preds: List[np.ndarray] = []
    for si, idx in enumerate(steps):
        feats = features(idx)
        ids = model.generate(feats, **gen_kwargs)
        ids = ids.to(comm_device) if comm_device is not None else ids
        ids = pad_across_processes(ids, pad_token_id)
        fid = torch.tensor(idx, dtype=torch.int64, device=ids.device)
        ids, fid = _all_gather_rows(ids), _all_gather_rows(fid)
        if si == len(steps) - 1 and rem > 0:
            ids, fid = ids[:rem], fid[:rem]
        eval_preds.extend(ids.cpu().numpy())
        eval_ids.extend(int(x) for x in fid.cpu().tolist())
        if on_step is not None:
            on_step(si, len(steps))
    return eval_ids, eval_preds


def write_transcription_csv(path: str, file_ids: Iterable[str], preds: Iterable[np.ndarray]) -> None:
    """``train-transcription.csv`` exactly as run_pseudo_labelling.py:347-350 writes it: a header row
    then ``[file_id, str(ndarray)]`` per item (numpy's default array repr of the token row)."""
    with open(path, "w", encoding="UTF8", newline="") as f:
        w = csv.writer(f)
        w.writerow(["file_id", "whisper_transcript"])
        w.writerows([[fid, p] for fid, p in zip(file_ids, preds)])

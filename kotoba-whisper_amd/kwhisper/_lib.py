"""ctypes binding of the kwhisper C ABI (include/kwhisper.h).

The shared library is built in-tree (``kotoba-whisper_amd/csrc/Makefile`` ->
``kwhisper/libkwhisper.so``).  There is no fallback: if the library is
missing or fails to load, every op raises.  torch is imported first so the
library binds to the HIP runtime torch already loaded (one runtime per
process; both carry SONAME libamdhip64.so.7).
"""
from __future__ import annotations

import ctypes
import threading
import weakref
import os

import torch  # noqa: F401  (must precede the library load: shared HIP runtime)

LIB_PATH = os.environ.get("KWHISPER_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libkwhisper.so")
# torch.ops.kw.* (csrc/torch_ops.cpp), linked against libkwhisper.so found beside it
TORCH_LIB_PATH = os.environ.get("KWHISPER_TORCH_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                                      "libkwhisper_torch.so")
TORCH_OPS = ("log_mel", "mel_to_time_major", "gemm", "dec_linear", "pack_weight", "layernorm", "attention", "embed",
             "self_attn_step", "dec_qkv_self", "dec_xq_cross", "cross_attn_step", "greedy_step", "dec_lm_greedy",
             "beam_logprobs", "beam_select")

KW_OK, KW_EINVAL, KW_EHIP, KW_EUNSUPPORTED = 0, 1, 2, 3
KW_DT_F32, KW_DT_BF16 = 0, 1
KW_EPI_STORE, KW_EPI_RESID, KW_EPI_HEADSPLIT = 0, 1, 2

c_i64 = ctypes.c_int64
c_i32 = ctypes.c_int32
c_vp = ctypes.c_void_p


class GemmArgs(ctypes.Structure):
    _fields_ = [
        ("dtype", ctypes.c_int), ("c_dtype", ctypes.c_int),
        ("A", c_vp), ("lda", c_i64), ("a_rows_per_batch", c_i64), ("a_batch_stride", c_i64),
        ("W", c_vp), ("bias", c_vp),
        ("C", c_vp), ("ldc", c_i64), ("c_rows_per_batch", c_i64), ("c_batch_stride", c_i64),
        ("M", c_i64), ("N", c_i64), ("K", c_i64),
        ("epilogue", ctypes.c_int), ("gelu", ctypes.c_int),
        ("scale", ctypes.c_float), ("scale_cols", c_i64),
        ("row_add", c_vp), ("row_add_period", c_i64),
        ("hs_seq", c_i64), ("hs_heads", c_i64), ("hs_head_dim", c_i64),
    ]


class DecLinearArgs(ctypes.Structure):
    _fields_ = [
        ("x", c_vp), ("ldx", c_i64), ("ln", ctypes.c_int), ("ln_eps", ctypes.c_float),
        ("ln_colsum", c_vp), ("W", c_vp), ("bias", c_vp), ("epilogue", ctypes.c_int),
        ("C", c_vp), ("ldc", c_i64), ("c_dtype", ctypes.c_int),
        ("gelu", ctypes.c_int), ("scale", ctypes.c_float), ("scale_cols", c_i64),
        ("h", c_vp), ("hb", c_vp), ("ldh", c_i64),
        ("M", c_i64), ("N", c_i64), ("K", c_i64),
        ("workspace", c_vp), ("ws_bytes", ctypes.c_size_t),
    ]


class QkvSelfArgs(ctypes.Structure):
    _fields_ = [
        ("x", c_vp), ("ldx", c_i64), ("ln_eps", ctypes.c_float), ("ln_colsum", c_vp), ("W", c_vp), ("bias", c_vp),
        ("scale", ctypes.c_float), ("M", c_i64), ("d", c_i64), ("H", c_i64), ("k_cache", c_vp), ("v_cache", c_vp),
        ("t_max", c_i64), ("cur_len", c_vp), ("out", c_vp), ("workspace", c_vp), ("ws_bytes", ctypes.c_size_t),
    ]


class XqCrossArgs(ctypes.Structure):
    _fields_ = [
        ("x", c_vp), ("ldx", c_i64), ("ln_eps", ctypes.c_float), ("ln_colsum", c_vp), ("W", c_vp), ("bias", c_vp),
        ("scale", ctypes.c_float), ("M", c_i64), ("d", c_i64), ("H", c_i64), ("k", c_vp), ("v", c_vp),
        ("S", c_i64), ("out", c_vp), ("workspace", c_vp), ("ws_bytes", ctypes.c_size_t),
    ]


class SamplerArgs(ctypes.Structure):
    _fields_ = [
        ("logits", c_vp), ("B", c_i64), ("V", c_i64),
        ("suppress_mask", c_vp), ("begin_suppress", c_vp), ("n_begin_suppress", c_i32),
        ("return_timestamps", c_i32),
        ("ts_begin", c_i32), ("no_ts_id", c_i32), ("eos_id", c_i32), ("pad_id", c_i32),
        ("max_initial_ts", c_i32),
        ("ids", c_vp), ("ids_stride", c_i64),
        ("cur_len", c_vp), ("max_length", c_i32), ("begin_index", c_i32),
        ("unfinished", c_vp), ("counter", c_vp), ("n_unfinished", c_vp), ("scores_out", c_vp),
        ("workspace", c_vp), ("ws_bytes", ctypes.c_size_t),
    ]


class BeamLogprobsArgs(ctypes.Structure):
    _fields_ = [
        ("logits", c_vp), ("R", c_i64), ("V", c_i64),
        ("suppress_mask", c_vp), ("begin_suppress", c_vp), ("n_begin_suppress", c_i32),
        ("return_timestamps", c_i32), ("ts_begin", c_i32), ("no_ts_id", c_i32), ("eos_id", c_i32),
        ("max_initial_ts", c_i32), ("ids", c_vp), ("ids_stride", c_i64), ("cur_len", c_vp),
        ("begin_index", c_i32), ("k", c_i32), ("cand_val", c_vp), ("cand_idx", c_vp), ("done", c_vp),
        ("workspace", c_vp), ("ws_bytes", ctypes.c_size_t),
    ]


class BeamSelectArgs(ctypes.Structure):
    _fields_ = [
        ("B", c_i64), ("num_beams", c_i32), ("V", c_i64), ("cand_val", c_vp), ("cand_idx", c_vp),
        ("ids", c_vp), ("ids_stride", c_i64), ("bp", c_vp), ("bp_stride", c_i64), ("run_scores", c_vp),
        ("fin_seq", c_vp), ("fin_stride", c_i64), ("fin_score", c_vp), ("fin_len", c_vp), ("fin_flag", c_vp),
        ("unsat", c_vp), ("cur_len", c_vp), ("begin_index", c_i32), ("max_length", c_i32), ("eos_id", c_i32),
        ("fill_id", c_i32), ("length_penalty", ctypes.c_float), ("early_stopping", c_i32),
        ("counter", c_vp), ("go", c_vp), ("done", c_vp), ("item_flags", c_vp),
    ]


EXPORTS = {
    "kw_version": (ctypes.c_int, []),
    "kw_stream_create": (ctypes.c_int, [ctypes.POINTER(c_vp)]),
    "kw_stream_destroy": (ctypes.c_int, [c_vp]),
    "kw_last_error": (ctypes.c_char_p, []),
    "kw_log_mel": (ctypes.c_int, [c_vp, c_i64, c_i64, c_i64, c_vp, ctypes.c_int, c_vp, c_vp, c_vp]),
    "kw_mel_to_time_major": (ctypes.c_int, [c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, ctypes.c_int, c_vp]),
    "kw_gemm": (ctypes.c_int, [ctypes.POINTER(GemmArgs), c_vp]),
    "kw_dec_linear": (ctypes.c_int, [ctypes.POINTER(DecLinearArgs), c_vp]),
    "kw_dec_linear_workspace_bytes": (ctypes.c_size_t, [c_i64, c_i64]),
    "kw_pack_weight": (ctypes.c_int, [c_vp, c_i64, c_i64, c_vp, c_vp]),
    "kw_packed_weight_bytes": (ctypes.c_size_t, [c_i64, c_i64]),
    "kw_layernorm": (ctypes.c_int, [c_vp, c_i64, c_i64, c_vp, c_vp, ctypes.c_float, c_vp, ctypes.c_int, c_vp, c_vp]),
    "kw_layernorm_bf16res": (ctypes.c_int, [c_vp, c_i64, c_i64, c_vp, c_vp, ctypes.c_float, c_vp, ctypes.c_int, c_vp,
                                            c_vp]),
    "kw_attention": (ctypes.c_int, [ctypes.c_int, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp]),
    "kw_embed": (ctypes.c_int, [ctypes.c_int, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp]),
    "kw_self_attn_step": (ctypes.c_int, [ctypes.c_int, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_i64, c_vp,
                                         c_vp, c_i64, c_vp, c_vp, ctypes.c_size_t, c_vp]),
    "kw_self_attn_workspace": (ctypes.c_size_t, [c_i64, c_i64, c_i64]),
    "kw_cross_attn_step": (ctypes.c_int, [ctypes.c_int, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_i64, c_vp,
                                          c_vp, ctypes.c_size_t, c_vp]),
    "kw_cross_attn_workspace": (ctypes.c_size_t, [c_i64, c_i64, c_i64, c_i64, c_i64]),
    "kw_dec_qkv_self": (ctypes.c_int, [ctypes.POINTER(QkvSelfArgs), c_vp]),
    "kw_dec_qkv_self_workspace": (ctypes.c_size_t, [c_i64, c_i64]),
    "kw_dec_qkv_self_supported": (ctypes.c_int, [c_i64, c_i64, c_i64]),
    "kw_dec_xq_cross": (ctypes.c_int, [ctypes.POINTER(XqCrossArgs), c_vp]),
    "kw_dec_xq_cross_workspace": (ctypes.c_size_t, [c_i64, c_i64, c_i64, c_i64]),
    "kw_dec_xq_cross_supported": (ctypes.c_int, [c_i64, c_i64, c_i64, c_i64]),
    "kw_cross_attn_pair_kernel": (ctypes.c_int, [c_i64, c_i64, ctypes.c_int]),
    "kw_dec_qkv_self_status_offset": (ctypes.c_size_t, [c_i64, c_i64]),
    "kw_dec_xq_cross_status_offset": (ctypes.c_size_t, [c_i64, c_i64, c_i64, c_i64]),
    "kw_cross_attn_status_offset": (ctypes.c_size_t, [c_i64, c_i64, c_i64, c_i64, c_i64]),
    "kw_greedy_step": (ctypes.c_int, [ctypes.POINTER(SamplerArgs), c_vp]),
    "kw_greedy_step_workspace": (ctypes.c_size_t, [c_i64]),
    "kw_dec_lm_greedy": (ctypes.c_int, [ctypes.POINTER(DecLinearArgs), ctypes.POINTER(SamplerArgs), c_vp]),
    "kw_dec_lm_greedy_workspace": (ctypes.c_size_t, [c_i64, c_i64]),
    "kw_dec_lm_greedy_supported": (ctypes.c_int, [c_i64, c_i64, c_i64]),
    "kw_beam_logprobs": (ctypes.c_int, [ctypes.POINTER(BeamLogprobsArgs), c_vp]),
    "kw_beam_logprobs_workspace": (ctypes.c_size_t, [c_i64]),
    "kw_beam_select": (ctypes.c_int, [ctypes.POINTER(BeamSelectArgs), c_vp]),
}

_lib = None


class KWError(RuntimeError):
    pass


def load(path: str = LIB_PATH):
    """Load and type the library once; raises if it is missing (no fallback path exists)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise KWError(
            f"kwhisper native library not found at {path}; build it with "
            "`make -C kotoba-whisper_amd/csrc` or `python -c 'import __graft_entry__ as g; g.build()'`"
        )
    lib = ctypes.CDLL(path)
    for name, (res, args) in EXPORTS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


_torch_ops = None


def load_torch_ops(path: str = TORCH_LIB_PATH):
    """Load the PyTorch custom-op library once and return ``torch.ops.kw``; raises if it is missing (no
    fallback path exists).  Registers fake (meta) implementations so torch.compile / export can trace the
    ops: each mutates its output tensors in place and returns nothing."""
    global _torch_ops
    if _torch_ops is not None:
        return _torch_ops
    if not os.path.exists(path):
        raise KWError(
            f"kwhisper torch-op library not found at {path}; build it with `make -C kotoba-whisper_amd/csrc` or "
            "`python -c 'import __graft_entry__ as g; g.build()'`"
        )
    load()  # the C ABI library first (same HIP runtime, its last-error state is shared)
    torch.ops.load_library(path)
    kw = torch.ops.kw
    for name in TORCH_OPS:
        try:
            torch.library.register_fake(f"kw::{name}")(lambda *a, **k: None)
        except RuntimeError:  # already registered (library re-loaded in this process)
            pass
    _torch_ops = kw
    return kw


def check(rc: int, what: str) -> None:
    if rc != KW_OK:
        msg = _lib.kw_last_error().decode(errors="replace") if _lib is not None else ""
        if rc == KW_EINVAL:
            raise ValueError(f"{what}: {msg}")
        raise KWError(f"{what} failed (code {rc}): {msg}")


_OWN_STREAMS = []  # (raw handle, torch stream): every stream made here, kept for the process's lifetime
_FREE_STREAMS = {}  # device index -> streams whose owner is gone, handed out again before a new one is made
# re-entrant: release_stream also runs from weakref.finalize callbacks, i.e. from whatever allocation on this thread
# triggers a garbage collection -- possibly inside new_stream's own locked section
_STREAM_LOCK = threading.RLock()


def new_stream(device=None, owner=None):
    """A torch stream over a HIP stream of its own (``kw_stream_create``), not one of PyTorch's pooled streams: a pool
    hands the same stream to two host threads once it wraps around, and a lane thread's launches on a stream that
    another lane's hipGraph capture has forked into would join that capture ("capturing stream has unjoined work").
    Every stream a capture uses or forks into comes from here.  Streams are recycled, never destroyed: ``owner``
    (an object) returns the stream when it is garbage collected, ``release_stream`` returns it explicitly; either
    way it is handed out again only after that -- so repeated calls (sessions, lanes, pipeline calls) reuse streams
    instead of making more."""
    import torch

    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    if dev.index is None:  # "cuda": the current device (free lists are keyed by index, as s.device.index)
        dev = torch.device("cuda", torch.cuda.current_device())
    free = _FREE_STREAMS.setdefault(dev.index, [])  # (allocation outside the lock; setdefault is atomic)
    with _STREAM_LOCK:
        s = free.pop() if free else None
    if s is None:
        h = ctypes.c_void_p()
        with torch.cuda.device(dev):
            check(load().kw_stream_create(ctypes.byref(h)), "kw_stream_create")
        s = torch.cuda.ExternalStream(h.value, device=dev)
        entry = (h, s)
        with _STREAM_LOCK:
            _OWN_STREAMS.append(entry)
    if owner is not None:
        weakref.finalize(owner, release_stream, s)
    return s


def release_stream(s) -> None:
    """Hand a ``new_stream`` stream back (its owner is done with it; work already queued on it stays ordered ahead of
    whatever its next user queues)."""
    free = _FREE_STREAMS.setdefault(s.device.index, [])
    with _STREAM_LOCK:
        free.append(s)

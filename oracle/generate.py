"""Oracle Whisper generate (greedy) -- TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

A pure-Python/numpy restatement of ``WhisperGenerationMixin.generate`` (transformers 5.15.0,
TF/models/whisper/generation_whisper.py), greedy and beam search:

  * prompt:       ``_retrieve_init_tokens``           :1455-1608 (+ ``detect_language`` :1620-1674)
  * processors:   ``_retrieve_logit_processors``       :1774-1812
                  SuppressTokens        TF/generation/logits_process.py:1869-1906
                  SuppressTokensAtBegin                                :1816-1866
                  WhisperTimeStamp                                     :1909-2047
  * seek loop:    ``generate``                          :785-903 (``_maybe_reduce_batch`` :1834,
                  ``_get_input_segment`` :1847, ``_set_max_new_tokens_and_length`` :1920-1946)
  * greedy:       ``GenerationMixin._sample``  TF/generation/utils.py:2783-2941 (argmax first-max,
                  finished rows -> pad :2929, MaxLength / EOS stopping ``stopping_criteria.py:75-77``)
  * beam search:  ``GenerationMixin._beam_search``  TF/generation/utils.py:3208-3527 with
                  ``_get_top_k_continuations`` :3077, ``_get_running_beams_for_next_iteration`` :3131,
                  ``_update_finished_beams`` :3153, ``_check_early_stop_heuristic`` :3008,
                  ``_beam_search_has_unfinished_sequences`` :3055; processors act on log-probs
                  (log_softmax first, :3380-3381); inputs expanded x num_beams
  * postprocess:  ``generate_with_fallback`` :1042-1086 (strip prompt, pad-count quirk, strip EOS),
                  ``_retrieve_segment`` :1977-2074, ``_pad_to_max_length`` :126-237 (right pad)
"""
from __future__ import annotations

import copy

import numpy as np

from .whisper_np import WhisperNP

def _lang_id(language, gen):
    """``language_to_id`` (generation_whisper.py:1464-1485) for codes and ``<|xx|>`` tokens."""
    lang = language.lower()
    tok = lang if lang in gen["lang_to_id"] else f"<|{lang}|>"
    if tok not in gen["lang_to_id"]:
        raise ValueError(f"Unsupported language: {lang}.")
    return gen["lang_to_id"][tok]


def init_tokens(gen: dict, batch_size: int, language, task, return_timestamps, detect=None):
    """``_retrieve_init_tokens`` (generation_whisper.py:1455-1608) for the task/language API."""
    tokens = [gen["decoder_start_token_id"]]
    langs = list(language) if isinstance(language, (list, tuple)) else ([language] if language is not None else [None] * batch_size)
    rows = [list(tokens) for _ in langs]
    lang_ids = None
    if language is not None:
        lang_ids = [_lang_id(l, gen) for l in langs]
    elif gen.get("lang_to_id") and detect is not None:
        lang_ids = list(detect())
    if lang_ids is not None:
        for i in range(len(rows)):
            if len(rows[i]) > 1:
                rows[i][1] = lang_ids[i]
            else:
                rows[i].append(lang_ids[i])
    for r in rows:
        if task is not None:
            r.append(gen["task_to_id"][task])
        elif language is not None:
            if not any(t in r for t in gen["task_to_id"].values()):
                r.append(gen["task_to_id"]["transcribe"])
        if not return_timestamps and r[-1] != gen["no_timestamps_token_id"]:
            r.append(gen["no_timestamps_token_id"])
        elif return_timestamps and r[-1] == gen["no_timestamps_token_id"]:
            r.pop()
    arr = np.asarray(rows, dtype=np.int64)
    return np.broadcast_to(arr, (batch_size, arr.shape[1])).copy()


def process_logits(input_ids: np.ndarray, scores: np.ndarray, gen: dict, begin_index: int,
                   return_timestamps: bool) -> np.ndarray:
    """Suppress -> SuppressAtBegin -> WhisperTimeStamp on f32 scores (B, V)."""
    s = scores.astype(np.float32).copy()
    ninf = np.float32(-np.inf)
    if gen.get("suppress_tokens"):
        s[:, np.asarray(gen["suppress_tokens"])] = ninf
    if gen.get("begin_suppress_tokens") and input_ids.shape[1] == begin_index:
        s[:, np.asarray(gen["begin_suppress_tokens"])] = ninf
    if return_timestamps:
        ts_begin = gen["no_timestamps_token_id"] + 1
        eos = gen["eos_token_id"]
        s[:, gen["no_timestamps_token_id"]] = ninf
        for k in range(input_ids.shape[0]):
            sampled = input_ids[k, begin_index:]
            seq = sampled.tolist()
            last_ts = len(seq) >= 1 and seq[-1] >= ts_begin
            pen_ts = len(seq) < 2 or seq[-2] >= ts_begin
            if last_ts:
                if pen_ts:
                    s[k, ts_begin:] = ninf
                else:
                    s[k, :eos] = ninf
            stamps = sampled[sampled >= ts_begin]
            if stamps.size > 0:
                last = stamps[-1] if (last_ts and not pen_ts) else stamps[-1] + 1
                s[k, ts_begin:last] = ninf
        if input_ids.shape[1] == begin_index:
            s[:, :ts_begin] = ninf
            mi = gen.get("max_initial_timestamp_index")
            if mi is not None:
                s[:, ts_begin + mi + 1:] = ninf
        m = s.max(-1, keepdims=True)
        with np.errstate(invalid="ignore", divide="ignore"):
            lse = m + np.log(np.exp(s - m).sum(-1, keepdims=True, dtype=np.float64)).astype(np.float32)
            logp = (s - lse).astype(np.float32)
            for k in range(s.shape[0]):
                lp = logp[k, ts_begin:].astype(np.float64)
                mm = lp.max()
                ts_lp = mm + np.log(np.exp(lp - mm).sum()) if np.isfinite(mm) else -np.inf
                if ts_lp > logp[k, :ts_begin].max():
                    s[k, :ts_begin] = ninf
    return s


def greedy(model: WhisperNP, enc: np.ndarray, prompt: np.ndarray, gen: dict, max_length: int,
           begin_index: int, return_timestamps: bool, record=None):
    """``GenerationMixin._sample`` greedy loop. Returns (B, L) ids including the prompt."""
    pad, eos = gen["pad_token_id"], gen["eos_token_id"]
    ids = prompt.copy()
    b = ids.shape[0]
    unfinished = np.ones(b, dtype=bool)
    cache = model.new_cache(enc)
    logits = model.decode(ids, cache)[:, -1]
    while True:
        scores = process_logits(ids, logits.astype(np.float32), gen, begin_index, return_timestamps)
        nxt = scores.argmax(-1).astype(np.int64)
        if record is not None:
            record.append((logits.copy(), scores))
        nxt = np.where(unfinished, nxt, pad)
        ids = np.concatenate([ids, nxt[:, None]], axis=1)
        done = np.full(b, ids.shape[1] >= max_length) | (nxt == eos)
        unfinished &= ~done
        if not unfinished.any():
            break
        logits = model.decode(nxt[:, None], cache)[:, -1]
    return ids


def _log_softmax(x: np.ndarray) -> np.ndarray:
    """torch.nn.functional.log_softmax in fp32: x - max - log(sum(exp(x - max)))."""
    x = x.astype(np.float32)
    m = x.max(-1, keepdims=True)
    lse = np.log(np.exp((x - m).astype(np.float64)).sum(-1, keepdims=True)).astype(np.float32)
    return ((x - m) - lse).astype(np.float32)


def _topk(x: np.ndarray, k: int) -> np.ndarray:
    """Indices of torch.topk(x, k) along the last axis (descending; ties -> lower index first)."""
    return np.argsort(-x, axis=-1, kind="stable")[..., :k]


def _take(a: np.ndarray, idx: np.ndarray) -> np.ndarray:
    """``_gather_beams`` (utils.py:2988): take_along_dim on axis 1."""
    while idx.ndim < a.ndim:
        idx = idx[..., None]
    return np.take_along_axis(a, idx, axis=1)


def beam_search(model: WhisperNP, enc: np.ndarray, prompt: np.ndarray, gen: dict, max_length: int,
                begin_index: int, return_timestamps: bool, num_beams: int, length_penalty: float = 1.0,
                early_stopping=False) -> np.ndarray:
    """``GenerationMixin._beam_search`` (utils.py:3208-3527), num_return_sequences = 1.
    Returns (B, prompt + generated) ids of the best beam per item, filled with pad_token_id."""
    f32 = np.float32
    NEG = f32(-1.0e9)
    pad, eos = gen["pad_token_id"], gen["eos_token_id"]
    B, P = prompt.shape
    nb = num_beams
    keep = 2 * nb  # max(2, 1 + n_eos) * num_beams with one EOS id (:3289)
    fill = pad if pad is not None else eos
    running = np.full((B, nb, max_length), fill, dtype=np.int64)
    running[:, :, :P] = prompt[:, None, :]
    sequences = running.copy()
    run_scores = np.zeros((B, nb), f32)
    run_scores[:, 1:] = NEG
    beam_scores = np.full((B, nb), NEG, f32)
    fin = np.zeros((B, nb), bool)
    unsat = np.ones((B, 1), bool)
    run_bi = np.full((B, nb, max_length - P), -1, np.int32)
    beam_idx = run_bi.copy()
    top_mask = np.arange(keep) < nb
    cache = model.new_cache(np.repeat(enc, nb, axis=0))
    logits = model.decode(np.repeat(prompt, nb, axis=0), cache)[:, -1]
    V = logits.shape[-1]
    cur_len = P
    while True:
        flat_hist = running.reshape(B * nb, max_length)[:, :cur_len]
        lp = process_logits(flat_hist, _log_softmax(logits), gen, begin_index, return_timestamps)
        lp = (lp.reshape(B, nb, V) + run_scores[:, :, None]).astype(f32).reshape(B, nb * V)
        # c. top-K continuations (:3077-3129)
        idx = _topk(lp, keep)
        topk_lp = np.take_along_axis(lp, idx, axis=1)
        cur_beam = idx // V
        tok = idx % V
        topk_bi = _take(run_bi, cur_beam).copy()
        topk_seq = _take(running, cur_beam).copy()
        topk_seq[:, :, cur_len] = tok
        topk_bi[:, :, cur_len - P] = cur_beam + np.arange(B)[:, None] * nb
        # d. stopping criteria: MaxLength on the new length, EOS on the new token
        hits = np.full((B, keep), cur_len + 1 >= max_length) | (tok == eos)
        # e. running beams (:3131-3151)
        trl = (topk_lp + hits.astype(f32) * NEG).astype(f32)
        nidx = _topk(trl, nb)
        running = _take(topk_seq, nidx)
        run_scores = np.take_along_axis(trl, nidx, axis=1)
        run_bi = _take(topk_bi, nidx)
        # f. finished beams (:3153-3205)
        did = hits & top_mask[None, :]
        tl = (topk_lp / f32((cur_len + 1 - P) ** length_penalty)).astype(f32)
        full = np.all(fin, axis=-1, keepdims=True) & (early_stopping is True)
        tl = tl + full.astype(f32) * NEG
        tl = tl + (~unsat).astype(f32) * NEG
        tl = (tl + (~did).astype(f32) * NEG).astype(f32)
        m_seq = np.concatenate([sequences, topk_seq], 1)
        m_scores = np.concatenate([beam_scores, tl], 1)
        m_bi = np.concatenate([beam_idx, topk_bi], 1)
        m_fin = np.concatenate([fin, did], 1)
        midx = _topk(m_scores, nb)
        sequences, beam_scores = _take(m_seq, midx), np.take_along_axis(m_scores, midx, axis=1)
        beam_idx, fin = _take(m_bi, midx), np.take_along_axis(m_fin, midx, axis=1)
        # g. cache reorder, early-stop heuristic (:3008-3053), loop condition (:3055-3075)
        model.reorder(cache, run_bi[..., cur_len - P].reshape(-1))
        cur_len += 1
        bhl = (max_length - P) if (early_stopping == "never" and length_penalty > 0.0) else (cur_len - P)
        best_run = (run_scores[:, :1] / f32(bhl ** length_penalty)).astype(f32)
        worst_fin = np.where(fin, beam_scores.min(1, keepdims=True), NEG)
        unsat = unsat & np.any(best_run > worst_fin, axis=-1, keepdims=True)
        go = unsat.any() and not (fin.all() and early_stopping is True) and not hits.all()
        if not go:
            break
        logits = model.decode(running.reshape(B * nb, max_length)[:, cur_len - 1: cur_len], cache)[:, -1]
    best_bi = beam_idx[:, 0]
    max_gen = int(((best_bi + 1) != 0).sum(1).max())
    return sequences[:, 0, : P + max_gen]


def _retrieve_segment(seq, ts_begin, seek_num_frames, time_offset, input_stride=2, time_precision=0.02,
                      time_precision_features=0.01):
    ts = seq >= ts_begin
    single_ending = ts[-2:].tolist() == [False, True]
    cons = np.where(ts[:-1] & ts[1:])[0] + 1
    if len(cons) > 0:
        slices = cons.tolist()
        if single_ending:
            slices.append(len(seq))
        else:
            slices[-1] += 1
        segs, last = [], 0
        for i, cur in enumerate(slices):
            is_last = i == len(slices) - 1
            st = seq[last:cur]
            start = int(st[0]) - ts_begin
            end = int(st[-1 if (not is_last or single_ending) else -2]) - ts_begin
            segs.append({"start": time_offset + start * time_precision, "end": time_offset + end * time_precision,
                         "tokens": st})
            last = cur
        if single_ending:
            offset = seek_num_frames
        else:
            offset = (int(seq[last - 2]) - ts_begin) * input_stride
    else:
        stamps = seq[ts]
        last_pos = int(seek_num_frames * time_precision_features / time_precision)
        if stamps.size > 0 and stamps[-1] != ts_begin:
            last_pos = float(stamps[-1] - ts_begin)
        segs = [{"start": time_offset, "end": time_offset + last_pos * time_precision, "tokens": seq}]
        offset = seek_num_frames
    return segs, offset


def generate(model: WhisperNP, input_features: np.ndarray, gen: dict, *, max_length=None, language=None,
             task=None, return_timestamps=None, attention_mask=None, return_dict_in_generate=False,
             return_segments=False, record=None, num_beams=1, length_penalty=1.0, early_stopping=False):
    """``WhisperGenerationMixin.generate`` restated: greedy (num_beams == 1) or beam search."""
    gen = copy.deepcopy(gen)
    feats = np.asarray(input_features, dtype=np.float32)
    b, _, total = feats.shape
    nseg = model.s.n_frames
    stride = 2
    shortform = total <= nseg
    if return_timestamps is None:
        return_timestamps = gen.get("return_timestamps", False)
    if not shortform:
        if return_timestamps is False:
            raise ValueError("long-form generation requires return_timestamps=True")
        return_timestamps = True
    if max_length is None:
        max_length = gen.get("max_length", 448)
    ts_begin = gen["no_timestamps_token_id"] + 1

    def detect():
        enc = model.encode(feats[:, :, :nseg])
        cache = model.new_cache(enc)
        lg = model.decode(np.full((b, 1), gen["decoder_start_token_id"]), cache)[:, -1]
        mask = np.ones(lg.shape[-1], dtype=bool)
        mask[list(gen["lang_to_id"].values())] = False
        lg[:, mask] = -np.inf
        return lg.argmax(-1)

    prompt_all = init_tokens(gen, b, language, task, return_timestamps, detect=detect)
    begin_index = prompt_all.shape[1]
    if not shortform and b > 1:
        if attention_mask is None:
            raise ValueError("batched long-form requires attention_mask")
        max_frames = np.asarray(attention_mask).sum(-1).astype(np.int64)
    else:
        max_frames = np.full(b, total, dtype=np.int64)
    seek = np.zeros(b, dtype=np.int64)
    segments = [[] for _ in range(b)]
    batch_map = list(range(b))
    cur_feats = feats
    last_outputs = None
    while (seek < max_frames).any():
        keep = [i for i, p in enumerate(batch_map) if seek[p] < max_frames[p]]
        cur_feats = cur_feats[keep]
        batch_map = [batch_map[i] for i in keep]
        time_offset = seek.astype(np.float64) * 0.02 / stride
        seek_num = np.minimum(max_frames - seek, nseg)
        seg_in = np.zeros((len(batch_map), feats.shape[1], nseg), dtype=np.float32)
        for i, p in enumerate(batch_map):
            sl = cur_feats[i, :, seek[p]: seek[p] + seek_num[p]]
            seg_in[i, :, : sl.shape[1]] = sl
        prompt = prompt_all[batch_map]
        max_length = min(max_length + min(model.s.max_target_positions // 2 - 1, prompt.shape[1]),
                         model.s.max_target_positions)
        enc = model.encode(seg_in)
        if num_beams > 1:
            ids = beam_search(model, enc, prompt, gen, max_length, prompt.shape[1], return_timestamps, num_beams,
                              length_penalty, early_stopping)
        else:
            ids = greedy(model, enc, prompt, gen, max_length, prompt.shape[1], return_timestamps, record)
        last_outputs = ids
        pad, eos = gen["pad_token_id"], gen["eos_token_id"]
        for i, p in enumerate(batch_map):
            seq = ids[i, prompt.shape[1]:]
            if seq[-1] == pad:
                n = int((seq == pad).sum())
                if pad == eos:
                    n -= 1
                if n != 0:
                    seq = seq[:-n]
            if seq[-1] == eos:
                seq = seq[:-1]
            segs, off = _retrieve_segment(seq, ts_begin, int(seek_num[p]), float(time_offset[p]), stride)
            seek[p] += off
            segments[p] += segs
    if return_dict_in_generate and not return_timestamps:
        return {"sequences": last_outputs}
    seqs = [np.concatenate([s["tokens"] for s in segs]) if segs else np.zeros(0, np.int64) for segs in segments]
    longest = max(len(s) for s in seqs)
    out = np.full((b, longest), gen["pad_token_id"], dtype=np.int64)
    for i, s in enumerate(seqs):
        out[i, : len(s)] = s
    if return_segments:
        return {"sequences": out, "segments": segments}
    return out

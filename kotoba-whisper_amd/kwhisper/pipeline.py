"""The ASR pipeline path on the MI355X engine.

kotoba-whisper's evaluation scripts reach the teacher through
``pipeline("automatic-speech-recognition", chunk_length_s=15, batch_size=...)`` (run_short_form_eval.py:110-117,
184-191; run_speed_eval.py:56-76).  ``ASRPipeline`` restates that path of transformers 5.15.0
(TF/pipelines/automatic_speech_recognition.py) for Whisper models, with the heavy parts on the GPU:

  * ``chunk_iter`` cuts each clip into ``chunk_len`` windows that overlap by ``stride_left`` /
    ``stride_right`` samples (:61-84; ``chunk_length_s / 6`` default stride, :432-447);
  * the chunks of every input are batched ``batch_size`` at a time, log-mel'd by the HIP feature
    extractor (zero-padded to 30 s, :67-72) and decoded by the drop-in ``generate`` (:483-560);
  * ``decode_asr`` merges the chunks' token streams exactly as the Whisper tokenizer's ``_decode_asr``
    does (TF/models/whisper/tokenization_whisper.py:901-1150): timestamp state machine, stride skips,
    the longest-common-sequence merge of overlapping windows (:1153-1270).

Text needs a vocabulary: with a tokenizer (anything with ``decode`` / ``all_special_ids`` /
``convert_tokens_to_ids``, e.g. a local ``WhisperTokenizer``) the output is HF's ``{"text": ...}``;
without one (no vocab files offline) the merged token ids are returned under ``"tokens"`` and every
text field holds token-id lists instead of strings.  Host code only: the per-chunk work is the engine's.
"""
from __future__ import annotations

import copy
from collections import defaultdict
from typing import Callable, Iterable, List, Optional, Sequence

import numpy as np
import torch

from . import _lib

from .config import LANGUAGES

__all__ = ["chunk_iter", "find_longest_common_sequence", "decode_asr", "ASRPipeline"]

_LANG_NAMES = dict(LANGUAGES)


def chunk_iter(n_samples: int, chunk_len: int, stride_left: int, stride_right: int):
    """Windows of a clip of ``n_samples`` samples (automatic_speech_recognition.py:61-84): yields
    ``(start, end, is_last, (chunk_samples, stride_left, stride_right))``.  A window is dropped when it
    is no longer than its left stride; the loop ends at the first window that reaches the clip's end."""
    step = chunk_len - stride_left - stride_right
    for start in range(0, n_samples, step):
        end = start + chunk_len
        n = min(end, n_samples) - start
        left = 0 if start == 0 else stride_left
        is_last = end >= n_samples
        right = 0 if is_last else stride_right
        if n > left:
            yield start, min(end, n_samples), is_last, (n, left, right)
        if is_last:
            break


def find_longest_common_sequence(sequences: Sequence[Sequence[int]]) -> List[int]:
    """Merge overlapping windows' token lists (tokenization_whisper.py:1153-1270, no token timestamps):
    for each next window, slide it over the running sequence, keep the alignment with the best
    ``matches / overlap + overlap / 1e4`` score (at least two matching tokens), and cut both halves at the
    middle of that overlap."""
    left = list(sequences[0])
    total: List[int] = []
    for right in sequences[1:]:
        right = list(right)
        ll, rl = len(left), len(right)
        best = 0.0
        cut = (ll, ll, 0, 0)
        la = np.asarray(left, dtype=np.int64)
        ra = np.asarray(right, dtype=np.int64)
        for i in range(1, ll + rl):
            eps = i / 10000.0
            l0, l1 = max(0, ll - i), min(ll, ll + rl - i)
            r0, r1 = max(0, i - ll), min(rl, i)
            matches = int(np.sum(la[l0:l1] == ra[r0:r1]))
            score = matches / i + eps
            if matches > 1 and score > best:
                best = score
                cut = (l0, l1, r0, r1)
        l0, l1, r0, r1 = cut
        total.extend(left[: (l1 + l0) // 2])
        left = right[(r1 + r0) // 2:]
    total.extend(left)
    return total


def _strip_prompt(ids: List[int], prompt_token_id: int, decoder_start_token_id: int) -> List[int]:
    """``WhisperTokenizer._strip_prompt`` (tokenization_whisper.py:725-741)."""
    if not ids or ids[0] != prompt_token_id:
        return ids
    return ids[ids.index(decoder_start_token_id):] if decoder_start_token_id in ids else []


def decode_asr(model_outputs, *, return_timestamps, return_language=None, time_precision: float,
               timestamp_begin: int, special_ids: Iterable[int], lang_of: dict, prompt_token_id: int,
               decoder_start_token_id: int, decode: Optional[Callable[[List[int]], str]] = None,
               segment_size: int = 1500):
    """The chunk merge of ``_decode_asr`` (tokenization_whisper.py:901-1150), segment-level timestamps.

    ``model_outputs``: per chunk, ``{"tokens": ids (1, T) or (T,), "stride": (chunk_s, left_s, right_s)}``
    (strides in seconds).  ``lang_of`` maps a language token id to its language name.  Returns
    ``(text, optional)`` as the reference does; with ``decode=None`` texts are token-id lists."""
    if return_timestamps == "word":
        raise NotImplementedError("word-level timestamps need cross-attention alignment heads (out of scope)")
    dec = decode if decode is not None else (lambda toks: list(toks))
    special = set(int(x) for x in special_ids)
    last_language = None

    def new_chunk():
        return {"language": last_language, "timestamp": [None, None], "text": "" if decode else []}

    chunks = []
    chunk = new_chunk()
    time_offset = 0.0
    previous_tokens: List[List[int]] = []
    skip = False
    right_stride_start = None
    for output in model_outputs:
        toks = output["tokens"]
        toks = toks.tolist() if hasattr(toks, "tolist") else list(toks)
        if toks and isinstance(toks[0], list):
            toks = toks[0]
        token_ids = _strip_prompt([int(t) for t in toks], prompt_token_id, decoder_start_token_id)
        last_timestamp = None
        first_timestamp = timestamp_begin
        cur_max_timestamp = 0.0
        prev_segments_len = 0.0
        penultimate_timestamp = 0.0
        if "stride" in output:
            chunk_len, stride_left, stride_right = output["stride"]
            time_offset -= stride_left
            right_stride_start = chunk_len - stride_right
            if stride_left:
                first_timestamp = stride_left / time_precision + timestamp_begin
            if stride_right:
                for token in reversed(token_ids):
                    if token >= timestamp_begin:
                        if last_timestamp is not None and (token - timestamp_begin) * time_precision < right_stride_start:
                            break
                        last_timestamp = token
        current_tokens: List[int] = []
        for i, token in enumerate(token_ids):
            if token in special:
                language = lang_of.get(token)
                if language is not None:
                    if last_language and language != last_language and not return_timestamps:
                        previous_tokens.append(current_tokens)
                        chunk["text"] = dec(find_longest_common_sequence(previous_tokens))
                        chunks.append(chunk)
                        previous_tokens = []
                        current_tokens = []
                        chunk = new_chunk()
                    chunk["language"] = language
                    last_language = language
            elif token >= timestamp_begin:
                timestamp = float((token - timestamp_begin) * time_precision)
                if timestamp < cur_max_timestamp:
                    last_was_single_ending = i >= 2 and not (
                        token_ids[i - 1] >= timestamp_begin and token_ids[i - 2] >= timestamp_begin)
                    if last_was_single_ending:
                        prev_segments_len += time_precision * segment_size
                    else:
                        cur_max_timestamp = penultimate_timestamp
                        prev_segments_len += penultimate_timestamp
                penultimate_timestamp = cur_max_timestamp
                cur_max_timestamp = timestamp
                time = round((token - timestamp_begin) * time_precision + time_offset + prev_segments_len, 2)
                if last_timestamp and token >= last_timestamp:
                    skip = True  # inside the right stride: resolved by the next window
                elif skip or (previous_tokens and token < first_timestamp):
                    skip = False
                elif chunk["timestamp"][0] is None:
                    chunk["timestamp"][0] = time
                elif time != chunk["timestamp"][0]:
                    chunk["timestamp"][1] = time
                    previous_tokens.append(current_tokens)
                    chunk["text"] = dec(find_longest_common_sequence(previous_tokens))
                    chunks.append(chunk)
                    previous_tokens = []
                    current_tokens = []
                    chunk = new_chunk()
            else:
                current_tokens.append(token)
        if "stride" in output:
            time_offset += chunk_len - stride_right
        if current_tokens:
            previous_tokens.append(current_tokens)
        elif not any(p for p in previous_tokens):
            chunk = new_chunk()
            previous_tokens = []
    if previous_tokens:
        chunk["text"] = dec(find_longest_common_sequence(previous_tokens))
        chunks.append(chunk)
    if decode is not None:
        full_text = "".join(c["text"] for c in chunks)
    else:
        full_text = [t for c in chunks for t in c["text"]]
    optional = {}
    if return_timestamps or return_language:
        for c in chunks:
            if not return_timestamps:
                c.pop("timestamp")
            else:
                c["timestamp"] = tuple(c["timestamp"])
            if not return_language:
                c.pop("language")
        optional = {"chunks": chunks}
    return full_text, optional


def _dist():
    import torch.distributed as dist

    return dist if dist.is_available() and dist.is_initialized() else None


def _check_same_inputs(dist, flat) -> None:
    """data_parallel splits the window batches over the ranks on the assumption that every rank holds the same
    windows: all-reduce (MAX of x and of -x) of the window count and of a digest of every window's item index,
    sample count and ALL its samples (sha256 over the whole window: edges alone match for silent or zero-padded
    starts and ends); raise on any difference (a per-rank shard of files would otherwise give position
    j the tokens of another rank's audio, or hang the gather on mismatched shapes).  sha256 runs at ~1 GB/s, i.e.
    about a millisecond per 15 s window, beside tens of milliseconds of decoding per window."""
    import hashlib

    h = hashlib.sha256()
    for i, c in flat:
        a = np.asarray(c["audio"].cpu() if torch.is_tensor(c["audio"]) else c["audio"], dtype=np.float32).reshape(-1)
        h.update(np.array([i, a.size], dtype=np.int64).tobytes())
        h.update(np.ascontiguousarray(a).tobytes())
    sig = [len(flat), int.from_bytes(h.digest()[:6], "little")]
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor(sig + [-x for x in sig], dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    hi, lo = t[:2].cpu().tolist(), [-x for x in t[2:].cpu().tolist()]
    if hi != lo:
        raise ValueError("ASRPipeline(data_parallel=True) needs the same inputs on every rank (window counts "
                         f"{lo[0]}..{hi[0]}, or the audio differs); shard the inputs yourself and use "
                         "data_parallel=False instead")


class ASRPipeline:
    """``pipeline("automatic-speech-recognition", model=<whisper>, chunk_length_s=..., batch_size=...)`` for
    the MI355X engine (TF/pipelines/automatic_speech_recognition.py, seq2seq_whisper path).

    ``model``: a ``KWhisperForConditionalGeneration``; ``feature_extractor``: ``kwhisper.WhisperFeatureExtractor``
    (built for the model's mel bins when omitted); ``tokenizer``: optional, for text output."""

    def __init__(self, model, feature_extractor=None, tokenizer=None, *, chunk_length_s: float = 0,
                 stride_length_s=None, batch_size: int = 1, generate_kwargs: Optional[dict] = None,
                 return_timestamps=None, data_parallel: bool = False, lanes: int = 1):
        from .feature_extraction import WhisperFeatureExtractor

        self.model = model
        self.feature_extractor = feature_extractor or WhisperFeatureExtractor(
            feature_size=model.config.num_mel_bins, device=model.device)
        self.tokenizer = tokenizer
        self.chunk_length_s = chunk_length_s
        self.stride_length_s = stride_length_s
        self.batch_size = max(1, int(batch_size))
        self.generate_kwargs = dict(generate_kwargs or {})
        self.return_timestamps = return_timestamps
        # data_parallel (opt-in) with a torch.distributed process group: every rank passes the SAME inputs, window
        # batches go round-robin over the ranks, one gather of the token matrices at the end, every rank returns the
        # full result (config 5 at W GPUs).  The ranks' inputs are checked to agree before the split
        # (_check_same_inputs); transformers' pipeline itself has no cross-rank behaviour, hence off by default
        self.data_parallel = bool(data_parallel)
        # lanes > 1: that many window batches decode at once on model.lane() handles (shared weights), one host
        # thread and stream each -- one batch's latency-bound decode chain beside another's HBM-bound
        # cross-attention (kwhisper.pseudo_label lanes); the output is the same
        if int(lanes) < 1:
            raise ValueError("lanes must be >= 1")
        if int(lanes) > 1 and not hasattr(model, "lane"):
            raise ValueError("lanes > 1 needs a model with lane() (an independent handle on the same weights)")
        self.lanes = int(lanes)
        self._lane_models = None
        self._lanes_run = set()  # lanes that have decoded a batch (their graphs captured) in an earlier call
        self.generation_config = self._pipeline_generation_config(model.generation_config)

    # the ASR pipeline's own generation defaults (TF/pipelines/automatic_speech_recognition.py:160-163)
    DEFAULT_MAX_NEW_TOKENS = 256
    DEFAULT_NUM_BEAMS = 5  # "follows openai's whisper implementation"

    @classmethod
    def _pipeline_generation_config(cls, model_gen):
        """The generation config the reference pipeline hands to every generate() call (TF/pipelines/base.py:
        886-907 via GenerationMixin._prepare_generation_config, TF/generation/utils.py): the pipeline defaults
        ``max_new_tokens=256, num_beams=5`` are the base and the model's generation config only fills fields
        they leave unset -- so the pipeline decodes with 5 beams (BASELINE config 5's beam=5) unless the call
        passes ``num_beams``; and ``max_new_tokens`` is dropped again when the model sets a non-default
        ``max_length`` (Whisper's 448), which then bounds the decode."""
        gen = model_gen.copy() if hasattr(model_gen, "copy") else copy.deepcopy(model_gen)
        gen.num_beams = cls.DEFAULT_NUM_BEAMS
        max_length = getattr(gen, "max_length", None)
        gen.pipeline_max_new_tokens = None if (max_length is not None and max_length != 20) else cls.DEFAULT_MAX_NEW_TOKENS
        return gen

    # ---- token vocabulary facts _decode_asr needs ------------------------------------------------------
    def _vocab(self):
        g = self.generation_config
        ts_begin = g.no_timestamps_token_id + 1
        if self.tokenizer is not None:
            tk = self.tokenizer
            special = list(tk.all_special_ids)
            ts_begin = tk.convert_tokens_to_ids("<|notimestamps|>") + 1
            prev = tk.convert_tokens_to_ids("<|startofprev|>")
            sot = tk.convert_tokens_to_ids("<|startoftranscript|>")
            lang_of = {}
            for t in special:
                name = _LANG_NAMES.get(tk.decode([t])[2:-2])
                if name is not None:
                    lang_of[t] = name
            return dict(timestamp_begin=ts_begin, special_ids=special, lang_of=lang_of, prompt_token_id=prev,
                        decoder_start_token_id=sot, decode=tk.decode)
        # the Whisper tokenizer's special ids: <|endoftext|> .. <|notimestamps|> (+ the pad id)
        special = list(range(g.eos_token_id, ts_begin)) + [g.pad_token_id]
        lang_of = {tid: _LANG_NAMES[tok[2:-2]] for tok, tid in g.lang_to_id.items()}
        return dict(timestamp_begin=ts_begin, special_ids=special, lang_of=lang_of,
                    prompt_token_id=g.prev_sot_token_id, decoder_start_token_id=g.decoder_start_token_id, decode=None)

    # ---- preprocess (:345-481) -------------------------------------------------------------------------
    def _chunks(self, inputs, chunk_length_s, stride_length_s):
        extra = {}
        if isinstance(inputs, dict):
            inputs = dict(inputs)
            stride = inputs.pop("stride", None)
            if not ("sampling_rate" in inputs and ("raw" in inputs or "array" in inputs)):
                raise ValueError(
                    "When passing a dictionary to AutomaticSpeechRecognitionPipeline, the dict needs to contain a "
                    '"raw" key containing the numpy array or torch tensor representing the audio and a "sampling_rate" '
                    "key, containing the sampling_rate associated with that array")
            raw = inputs.pop("raw", None)
            if raw is None:
                inputs.pop("path", None)  # a `datasets` audio dict's path is not carried along (:391-393)
                raw = inputs.pop("array", None)
            sr = inputs.pop("sampling_rate")
            extra = inputs
            if sr != self.feature_extractor.sampling_rate:
                raise ImportError("resampling needs torchaudio, which this build does not use: pass "
                                  f"{self.feature_extractor.sampling_rate} Hz audio")
            if stride is not None:
                raise ValueError("Stride is only usable with CTC models, try removing it !")
            inputs = raw
        if isinstance(inputs, torch.Tensor):
            inputs = inputs.detach().cpu().numpy()
        if not isinstance(inputs, np.ndarray):
            raise TypeError(f"We expect a numpy ndarray or torch tensor as input, got `{type(inputs)}`")
        if inputs.ndim != 1:
            inputs = inputs.mean(axis=0)
        sr = self.feature_extractor.sampling_rate
        if chunk_length_s:
            if stride_length_s is None:
                stride_length_s = chunk_length_s / 6
            if isinstance(stride_length_s, (int, float)):
                stride_length_s = [stride_length_s, stride_length_s]
            chunk_len = int(round(chunk_length_s * sr))
            sl = int(round(stride_length_s[0] * sr))
            sr_ = int(round(stride_length_s[1] * sr))
            if chunk_len < sl + sr_:
                raise ValueError("Chunk length must be superior to stride length")
            out = [dict(audio=inputs[a:b], is_last=last, stride=st, **extra)
                   for a, b, last, st in chunk_iter(inputs.shape[0], chunk_len, sl, sr_)]
        else:
            # one item; longer than 30 s -> Whisper long-form (seek loop in generate, :449-458)
            out = [dict(audio=inputs, is_last=True, **extra)]
        return out

    def _batch_features(self, audios):
        """Each item through the feature extractor as the reference's preprocess does (<= 30 s: padded to
        30 s; longer: truncation=False, padding="longest", :449-470), then the batch collated as its
        pad_collate_fn does: features right-padded with the extractor's padding value to the longest item,
        attention masks with zeros."""
        fe = self.feature_extractor
        if all(len(x) <= fe.n_samples for x in audios):
            f = fe(audios, sampling_rate=fe.sampling_rate, return_attention_mask=True)
            return f["input_features"], f["attention_mask"]
        items = []
        for x in audios:
            if len(x) > fe.n_samples:
                items.append(fe([x], sampling_rate=fe.sampling_rate, truncation=False, padding="longest",
                                return_attention_mask=True))
            else:
                items.append(fe([x], sampling_rate=fe.sampling_rate, return_attention_mask=True))
        T = max(f["input_features"].shape[-1] for f in items)
        n_mels = items[0]["input_features"].shape[1]
        feats = torch.full((len(items), n_mels, T), float(fe.padding_value), device=fe.device)
        mask = torch.zeros((len(items), T), dtype=torch.int32, device=fe.device)
        for i, f in enumerate(items):
            t = f["input_features"].shape[-1]
            feats[i, :, :t] = f["input_features"][0]
            mask[i, : f["attention_mask"].shape[-1]] = f["attention_mask"][0]
        return feats, mask

    def _decode_one(self, model, batch, gk):
        feats, mask = self._batch_features([c["audio"] for _, c in batch])
        out = model.generate(feats, attention_mask=mask, **gk)
        ids = out["sequences"] if isinstance(out, dict) else out
        return ids.cpu().numpy()

    def _decode_batches(self, batches, gk):
        """generate() over the window batches, in order: on the model alone, or (lanes > 1) batch j on lane j % n,
        a lane's first batch ever alone first (its graphs captured before the threads overlap), then one thread and
        stream per lane."""
        n = min(self.lanes, max(1, len(batches)))
        if n == 1:
            return [self._decode_one(self.model, b, gk) for b in batches]
        if self._lane_models is None or len(self._lane_models) < n:
            self._lane_models = [self.model] + [self.model.lane() for _ in range(n - 1)]
        models = self._lane_models[:n]
        local = [None] * len(batches)
        first = {}  # lane -> its first batch index for the threads
        for i in range(n):
            if i in self._lanes_run:
                first[i] = i
            else:
                local[i] = self._decode_one(models[i], batches[i], gk)
                self._lanes_run.add(i)
                first[i] = i + n
        import contextlib
        import threading

        streams = [_lib.new_stream(torch.cuda.current_device()) for _ in range(n)] \
            if torch.cuda.is_available() else [None] * n
        errs = []

        def work(i):
            try:
                with torch.cuda.stream(streams[i]) if streams[i] is not None else contextlib.nullcontext():
                    for j in range(first[i], len(batches), n):
                        local[j] = self._decode_one(models[i], batches[j], gk)
            except BaseException as e:  # re-raised on the calling thread
                errs.append(e)

        threads = [threading.Thread(target=work, args=(i,)) for i in range(n)]
        for th in threads:
            th.start()
        for th in threads:
            th.join()
        for st in streams:  # (recycled by the next call's lanes: _lib.new_stream)
            if st is not None:
                _lib.release_stream(st)
        if errs:
            raise errs[0]
        return local

    # ---- forward (:483-560) + postprocess (:600-710) -----------------------------------------------------
    def __call__(self, inputs, *, chunk_length_s=None, stride_length_s=None, return_timestamps=None,
                 return_language=None, generate_kwargs: Optional[dict] = None, batch_size: Optional[int] = None,
                 **kwargs):
        single = not isinstance(inputs, (list, tuple))
        items = [inputs] if single else list(inputs)
        cl = self.chunk_length_s if chunk_length_s is None else chunk_length_s
        sl = self.stride_length_s if stride_length_s is None else stride_length_s
        gk = dict(self.generate_kwargs)
        gk.update(generate_kwargs or {})
        gk.update(kwargs)
        rt = self.return_timestamps if return_timestamps is None else return_timestamps
        rt = rt or getattr(self.generation_config, "return_timestamps", False)
        if rt == "char":
            raise ValueError("Whisper cannot return `char` timestamps, only word level or segment level timestamps. "
                             "Use `return_timestamps='word'` or `return_timestamps=True` respectively.")
        if rt == "word":
            raise NotImplementedError("word-level timestamps are not supported by the MI355X engine")
        bs = self.batch_size if batch_size is None else max(1, int(batch_size))
        per_item = [self._chunks(x, cl, sl) for x in items]
        flat = [(i, c) for i, chs in enumerate(per_item) for c in chs]
        if rt:
            gk["return_timestamps"] = True
        gk.setdefault("generation_config", self.generation_config)
        mnt = getattr(gk["generation_config"], "pipeline_max_new_tokens", None)
        if mnt is not None and "max_length" not in gk and "max_new_tokens" not in gk:
            gk["max_new_tokens"] = mnt
        fe = self.feature_extractor
        tokens = [None] * len(flat)
        starts = list(range(0, len(flat), bs))
        dist = _dist() if self.data_parallel else None
        if dist is not None:
            _check_same_inputs(dist, flat)
        world, rank = (dist.get_world_size(), dist.get_rank()) if dist is not None else (1, 0)
        mine = starts[rank::world]  # data parallel: window batch j on rank j % W, no collective until the end
        local = self._decode_batches([flat[b0: b0 + bs] for b0 in mine], gk)
        if dist is not None:  # one exchange: every rank's window batches as generate() returned them
            from .pseudo_label import gather_matrices

            per_rank = gather_matrices(local, (len(starts) + world - 1) // world, int(self.generation_config.pad_token_id))
            local = [per_rank[j % world][j // world] for j in range(len(starts))]
        for b0, ids in zip(starts if dist is not None else mine, local):
            ids = torch.from_numpy(np.ascontiguousarray(ids))
            for j in range(ids.shape[0]):
                tokens[b0 + j] = ids[j: j + 1]
        vocab = self._vocab()
        time_precision = fe.chunk_length / self.model.config.max_source_positions
        results = []
        k = 0
        for chs in per_item:
            outputs = []
            for c in chs:
                o = {"tokens": tokens[k]}
                k += 1
                if "stride" in c:
                    n, left, right = c["stride"]
                    o["stride"] = (n / fe.sampling_rate, left / fe.sampling_rate, right / fe.sampling_rate)
                outputs.append(o)
            text, optional = decode_asr(outputs, return_timestamps=rt, return_language=return_language,
                                        time_precision=time_precision, **vocab)
            extra = defaultdict(list)
            for c in chs:
                for key, v in c.items():
                    if key not in ("audio", "is_last", "stride"):
                        extra[key].append(v)
            res = {"text": text, **optional, **extra} if vocab["decode"] is not None else \
                {"text": None, "tokens": text, **optional, **extra}
            results.append(res)
        return results[0] if single else results

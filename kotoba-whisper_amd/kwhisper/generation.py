"""HF-compatible drop-in: ``WhisperForConditionalGeneration.generate()`` on the MI355X engine.

The object returned by ``from_pretrained``/``from_state_dict`` is what the reference passes as
``model`` at run_pseudo_labelling.py:338 (and v3 :313-318) and what the ASR pipeline's ``_forward``
calls at TF/pipelines/automatic_speech_recognition.py:529.  It keeps HF's call signature,
argument meaning, errors and token output (transformers 5.15.0,
TF/models/whisper/generation_whisper.py:383-968):

  * prompt ``[sot, lang, task(, notimestamps)]``                     :1455-1608
  * language detection when ``language`` is None (multilingual)      :1620-1674
  * processors Suppress -> SuppressAtBegin -> TimeStamp (on device)  :1774-1812
  * the seek loop with the cumulative ``max_length`` growth          :785-903, :1920-1946
  * strip prompt / pad-count quirk / strip EOS                       :1042-1086
  * segments and right padding with ``pad_token_id``                 :1977-2074, :126-237
  * ``return_dict_in_generate`` (no timestamps): sequences incl. prompt  :916-934
  * ``num_beams`` > 1: GenerationMixin._beam_search on device (TF/generation/utils.py:3208-3527)
"""
from __future__ import annotations

import copy
import os
from dataclasses import dataclass

import numpy as np
import torch

from .config import PRESETS, GenerationConstants, WhisperShape, generation_constants, language_to_id
from .engine import WhisperEngine

_SUPPORTED = {
    "generation_config", "logits_processor", "stopping_criteria", "return_timestamps", "task", "language",
    "is_multilingual", "attention_mask", "max_length", "max_new_tokens", "num_beams", "return_dict_in_generate",
    "return_segments", "encoder_outputs", "prompt_ids", "temperature", "do_sample", "condition_on_prev_tokens",
    "compression_ratio_threshold", "logprob_threshold", "no_speech_threshold", "return_token_timestamps",
    "output_scores", "output_logits", "time_precision", "time_precision_features", "num_segment_frames",
    "synced_gpus", "force_unique_generate_call", "prefix_allowed_tokens_fn", "prompt_condition_type",
    "monitor_progress", "use_cache", "num_return_sequences", "length_penalty", "early_stopping",
}


@dataclass
class ModelConfig:
    """The ``model.config`` fields callers read (run_pseudo_labelling.py:233,295)."""

    shape: WhisperShape

    def __getattr__(self, k):
        return getattr(self.shape, k)


class EncoderOutput:
    def __init__(self, h):
        self.last_hidden_state = h

    def __getitem__(self, i):
        if i == 0:
            return self.last_hidden_state
        raise IndexError(i)


class _Encoder:
    """``model.get_encoder()``: returns (B, 1500, d) last_hidden_state (modeling_whisper.py:592-646)."""

    def __init__(self, eng):
        self.eng = eng

    def __call__(self, input_features, **kw):
        B = input_features.shape[0]
        h = self.eng.encode(input_features)
        return EncoderOutput(h.view(B, self.eng.shape.max_source_positions, self.eng.shape.d_model))


class KWhisperForConditionalGeneration:
    main_input_name = "input_features"

    def __init__(self, engine: WhisperEngine):
        self.engine = engine
        self.config = ModelConfig(engine.shape)
        self.generation_config = engine.generation_config
        self._sessions = {}
        self.stats = {}
        # True: generate() also keeps every seek pass's decoded ids in stats["pass_ids"] (validation: a fixture of the
        # engine's own multi-pass trajectory, tools/dump_hipmel.py)
        self.record_pass_ids = False
        self._memo = None  # generate_multitask's per-batch encoder memo
        self._memo_count = 0

    # ---- nn.Module-ish surface used by callers ---------------------------------------------------
    @property
    def device(self):
        return self.engine.device

    @property
    def dtype(self):
        return self.engine.dtype

    def eval(self):
        return self

    def to(self, *a, **k):
        return self

    def get_encoder(self):
        return _Encoder(self.engine)

    def lane(self) -> "KWhisperForConditionalGeneration":
        """An independent handle on the same weights (WhisperEngine.lane(): own activation buffers, streams and decode
        sessions) for running another batch at the same time from another host thread."""
        other = type(self)(self.engine.lane())
        other.generation_config = copy.deepcopy(self.generation_config)
        return other

    @classmethod
    def from_state_dict(cls, shape, state_dict, *, dtype=torch.bfloat16, device="cuda", generation_config=None):
        shape = PRESETS[shape] if isinstance(shape, str) else shape
        return cls(WhisperEngine(shape, state_dict, dtype=dtype, device=device, generation_config=generation_config))

    @classmethod
    def from_pretrained(cls, path_or_name, *, torch_dtype=torch.bfloat16, device="cuda", **kw):
        """Load a local HF checkpoint directory (config.json + *.safetensors).  No network access."""
        import json

        from safetensors.numpy import load_file

        if not os.path.isdir(path_or_name):
            raise OSError(f"{path_or_name} is not a local checkpoint directory (no hub access in this build)")
        cfg = json.load(open(os.path.join(path_or_name, "config.json")))
        shape = WhisperShape(
            name=cfg.get("_name_or_path", path_or_name), vocab_size=cfg["vocab_size"], num_mel_bins=cfg["num_mel_bins"],
            d_model=cfg["d_model"], encoder_layers=cfg["encoder_layers"],
            encoder_attention_heads=cfg["encoder_attention_heads"], encoder_ffn_dim=cfg["encoder_ffn_dim"],
            decoder_layers=cfg["decoder_layers"], decoder_attention_heads=cfg["decoder_attention_heads"],
            decoder_ffn_dim=cfg["decoder_ffn_dim"], max_source_positions=cfg.get("max_source_positions", 1500),
            max_target_positions=cfg.get("max_target_positions", 448),
            decoder_start_token_id=cfg.get("decoder_start_token_id", 50258), pad_token_id=cfg.get("pad_token_id", 50256),
            eos_token_id=cfg.get("eos_token_id", 50257), bos_token_id=cfg.get("bos_token_id", 50257))
        sd = {}
        for f in sorted(os.listdir(path_or_name)):
            if f.endswith(".safetensors"):
                sd.update(load_file(os.path.join(path_or_name, f)))
        gen = generation_constants(shape)
        gpath = os.path.join(path_or_name, "generation_config.json")
        if os.path.exists(gpath):
            gj = json.load(open(gpath))
            for k, v in gj.items():
                if hasattr(gen, k):
                    setattr(gen, k, v)
        return cls.from_state_dict(shape, sd, dtype=torch_dtype, device=device, generation_config=gen)

    # ---- generate ---------------------------------------------------------------------------------
    def _session(self, B, beams=1):
        key = (B, beams)
        if key not in self._sessions:
            self._sessions[key] = self.engine.new_session(B, beams=beams)
        return self._sessions[key]

    def generate(self, input_features=None, generation_config=None, logits_processor=None, stopping_criteria=None,
                 return_timestamps=None, task=None, language=None, is_multilingual=None, attention_mask=None,
                 return_dict_in_generate=None, return_segments=False, **kwargs):
        unknown = [k for k in kwargs if k not in _SUPPORTED]
        if unknown:
            raise ValueError(
                f"The following `model_kwargs` are not used by the model: {unknown} (note: typos in the generate "
                "arguments will also show up in this list)"
            )
        if logits_processor or stopping_criteria:
            raise NotImplementedError("custom logits_processor / stopping_criteria are not supported on device")
        for k in ("prompt_ids", "prefix_allowed_tokens_fn", "compression_ratio_threshold", "logprob_threshold",
                  "no_speech_threshold", "return_token_timestamps", "assistant_model"):
            if kwargs.get(k) is not None and kwargs.get(k) is not False:
                raise NotImplementedError(f"`{k}` is not supported by the MI355X engine yet")
        if kwargs.get("temperature") not in (None, 0, 0.0) or kwargs.get("do_sample"):
            raise NotImplementedError("sampling / temperature fallback is not supported (greedy and beam only)")
        if kwargs.get("num_return_sequences") not in (None, 1):
            raise NotImplementedError("num_return_sequences > 1 is not supported")
        gen: GenerationConstants = copy.deepcopy(generation_config or self.generation_config)
        if isinstance(gen, dict):
            gen = GenerationConstants(**gen)
        num_beams = kwargs.get("num_beams", gen.num_beams or 1)
        if num_beams > 8:
            raise NotImplementedError("num_beams > 8 is not supported by the device beam search")
        length_penalty = kwargs.get("length_penalty", getattr(gen, "length_penalty", 1.0))
        early_stopping = kwargs.get("early_stopping", getattr(gen, "early_stopping", False))
        max_new_tokens = kwargs.get("max_new_tokens")
        max_length = kwargs.get("max_length", gen.max_length)
        s = self.engine.shape
        eng = self.engine

        enc_given = kwargs.get("encoder_outputs")
        if input_features is None and enc_given is None:
            raise ValueError("Make sure to provide either `input_features` or `encoder_outputs` to `generate`.")
        if input_features is not None:
            feats = input_features.to(device=eng.device, dtype=torch.float32)
            B, total = feats.shape[0], feats.shape[-1]
        else:
            eh = enc_given.last_hidden_state if hasattr(enc_given, "last_hidden_state") else enc_given[0] \
                if isinstance(enc_given, (tuple, list)) else enc_given
            B, total = eh.shape[0], eh.shape[1] * 2
            feats = None
        nseg = s.n_frames
        shortform = total <= nseg
        if return_timestamps is None:
            return_timestamps = bool(getattr(gen, "return_timestamps", False))
        if not shortform:
            if return_timestamps is False:
                raise ValueError(
                    "You have passed more than 3000 mel input features (> 30 seconds) which automatically enables "
                    "long-form generation which requires the model to predict timestamp tokens. Please either pass "
                    "`return_timestamps=True` or make sure to pass no more than 3000 mel input features.")
            return_timestamps = True
        if return_dict_in_generate is None:
            return_dict_in_generate = False
        if is_multilingual is not None:
            gen.is_multilingual = is_multilingual
        if not gen.is_multilingual and (task is not None or language is not None):
            raise ValueError("Cannot specify `task` or `language` for an English-only model.")

        # prompt (init tokens)
        prompt_all = self._init_tokens(gen, B, language, task, return_timestamps, feats, enc_given)
        P = prompt_all.shape[1]

        if max_new_tokens is not None and max_new_tokens + P > s.max_target_positions:
            raise ValueError(
                f"The length of `decoder_input_ids`, including special start tokens, prompt tokens, and previous "
                f"tokens, is {P},  and `max_new_tokens` is {max_new_tokens}. Thus, the combined length of "
                f"`decoder_input_ids` and `max_new_tokens` is: {max_new_tokens + P}. This exceeds the "
                f"`max_target_positions` of the Whisper model: {s.max_target_positions}. You should either reduce "
                "the length of your prompt, or reduce the value of `max_new_tokens`, so that their combined length "
                f"is less than {s.max_target_positions}.")
        if not shortform and B > 1:
            if attention_mask is None:
                raise ValueError(
                    "When doing batched long-form audio transcription, make sure to pass an `attention_mask`. You "
                    "can retrieve the `attention_mask` by doing `processor(audio, ..., return_attention_mask=True)` ")
            max_frames = attention_mask.sum(-1).cpu().long().numpy()
        else:
            max_frames = np.full(B, total, dtype=np.int64)
        seek = np.zeros(B, dtype=np.int64)
        ts_begin = gen.timestamp_begin
        segments = [[] for _ in range(B)]
        batch_map = list(range(B))
        last_ids = None
        passes = 0
        row_passes = np.zeros(B, dtype=np.int64)
        pass_log, pass_ids = [], []  # per pass: (rows, their seek, their frame count); the decoded ids
        while (seek < max_frames).any():
            batch_map = [p for p in batch_map if seek[p] < max_frames[p]]
            cur = len(batch_map)
            row_passes[batch_map] += 1
            time_offset = seek.astype(np.float64) * 0.02 / 2
            seek_num = np.minimum(max_frames - seek, nseg)
            if feats is not None:
                whole = shortform and total == nseg and all(seek[p] == 0 for p in batch_map) and cur == B
                if whole:
                    seg_in = feats
                else:
                    seg_in = torch.zeros((cur, feats.shape[1], nseg), device=eng.device, dtype=torch.float32)
                    for i, p in enumerate(batch_map):
                        n = int(seek_num[p])
                        seg_in[i, :, :n] = feats[p, :, int(seek[p]): int(seek[p]) + n]
                enc_key = None
                memo = self._memo
                if memo is not None and whole and passes == 0:
                    # multi-task reuse: the first pass of every prompt sees the same mel, so the encoder and
                    # the cross-K/V projection run once per batch (clone: later passes reuse the buffer)
                    if "enc" not in memo:
                        memo["enc"] = eng.encode(seg_in).clone()
                    enc, enc_key = memo["enc"], ("memo", memo["id"])
                else:
                    enc = eng.encode(seg_in)
            else:
                if passes > 0:
                    raise NotImplementedError("encoder_outputs with a multi-pass seek loop")
                enc = eh.to(eng.device, eng.dtype).reshape(B * s.max_source_positions, s.d_model).contiguous()
                enc_key = None
            prompt = prompt_all[batch_map]
            if max_new_tokens is None:
                max_length = min(max_length + min(s.max_target_positions // 2 - 1, P), s.max_target_positions)
                eff_max = max_length
            else:
                eff_max = P + max_new_tokens
            sess = self._session(cur, num_beams)
            sess.set_encoder_output(enc, key=enc_key)
            if num_beams > 1:
                ids = sess.generate_beam(torch.from_numpy(prompt), gen, num_beams=num_beams, max_length=eff_max,
                                         return_timestamps=return_timestamps, length_penalty=length_penalty,
                                         early_stopping=early_stopping)
            else:
                ids = sess.generate(torch.from_numpy(prompt), gen, max_length=eff_max,
                                    return_timestamps=return_timestamps)
            passes += 1
            last_ids = ids
            pass_log.append(([int(p) for p in batch_map], [int(seek[p]) for p in batch_map],
                             [int(seek_num[p]) for p in batch_map]))
            if self.record_pass_ids:
                pass_ids.append(np.asarray(ids).copy())
            pad, eos = gen.pad_token_id, gen.eos_token_id
            for i, p in enumerate(batch_map):
                seq = ids[i, P:]
                if seq.size and seq[-1] == pad:
                    n = int((seq == pad).sum())
                    if pad == eos:
                        n -= 1
                    if n != 0:
                        seq = seq[:-n]
                if seq.size and seq[-1] == eos:
                    seq = seq[:-1]
                segs, off = _retrieve_segment(seq, ts_begin, int(seek_num[p]), float(time_offset[p]))
                seek[p] += off
                segments[p] += segs
        self.stats = {"passes": passes, "row_passes": row_passes, "pass_log": pass_log}
        if self.record_pass_ids:
            self.stats["pass_ids"] = pass_ids
        if return_dict_in_generate and not return_timestamps:
            return {"sequences": torch.from_numpy(last_ids).to(eng.device)}
        seqs = [np.concatenate([x["tokens"] for x in segs]) if segs else np.zeros(0, np.int64) for segs in segments]
        longest = max(len(x) for x in seqs) if seqs else 0
        out = np.full((B, longest), gen.pad_token_id, dtype=np.int64)
        for i, x in enumerate(seqs):
            out[i, : len(x)] = x
        res = torch.from_numpy(out).to(eng.device)
        if return_segments or (return_dict_in_generate and return_timestamps):
            return {"sequences": res, "segments": segments}
        return res

    def generate_multitask(self, input_features, tasks, **kwargs):
        """``generate`` once per (language, task) of ``tasks`` on the same features -- the inner loop of
        run_pseudo_labelling_v3.py:309-318 -- with ONE encoder pass and ONE cross-K/V projection shared by
        every prompt.  Each result is exactly what ``generate(input_features,
        language=..., task=..., **kwargs)`` returns on its own; only passes after the first (the
        timestamp seek loop's re-encodes of shifted mel) run the encoder again."""
        if not tasks:
            return []
        for k in ("language", "task", "encoder_outputs"):
            if k in kwargs:
                raise ValueError(f"generate_multitask takes `{k}` from `tasks`, not as a keyword")
        self._memo_count += 1
        self._memo = {"id": self._memo_count}
        try:
            return [self.generate(input_features, language=lang, task=task, **kwargs) for lang, task in tasks]
        finally:
            self._memo = None

    # ---- helpers ------------------------------------------------------------------------------------
    def detect_language(self, input_features=None, encoder_outputs=None, generation_config=None):
        """``detect_language`` (generation_whisper.py:1620-1674)."""
        gen = generation_config or self.generation_config
        eng = self.engine
        if input_features is not None:
            B = input_features.shape[0]
            enc = eng.encode(input_features[:, :, : eng.shape.n_frames].to(eng.device, torch.float32))
        else:
            eh = encoder_outputs.last_hidden_state if hasattr(encoder_outputs, "last_hidden_state") else encoder_outputs
            B = eh.shape[0]
            enc = eh.to(eng.device, eng.dtype).reshape(B * eng.shape.max_source_positions, eng.shape.d_model)
        sess = self._session(B)
        sess.set_encoder_output(enc)
        prompt = torch.full((B, 1), gen.decoder_start_token_id, dtype=torch.int64, device=eng.device)
        logits = sess.forward_logits(prompt).clone()
        mask = torch.ones(logits.shape[-1], dtype=torch.bool, device=logits.device)
        mask[list(gen.lang_to_id.values())] = False
        logits[:, mask] = -float("inf")
        return logits.argmax(-1)

    def _init_tokens(self, gen, B, language, task, return_timestamps, feats, enc_given):
        """``_retrieve_init_tokens`` (generation_whisper.py:1455-1608) for the task/language API."""
        if language is None and getattr(gen, "language", None) is not None:
            language = gen.language
        if task is None and getattr(gen, "task", None) is not None:
            task = gen.task
        if isinstance(language, (list, tuple)):
            if any(x is None for x in language):
                raise TypeError("Expected `language` to be `None`, a single string (e.g. `'en'`), or a list of "
                                "strings with length equal to the batch size (e.g. `('en', 'fr')` for a batch size "
                                "of 2). Got a list containing `None`.")
            if len(language) != B:
                raise ValueError("When passing a list of languages, the length of the list must match the batch "
                                 f"size. Expected length of {B}, but got {len(language)} languages.")
            langs = list(language)
        elif language is None:
            langs = [None] * B
        else:
            langs = [language]
        rows = [[gen.decoder_start_token_id] for _ in langs]
        lang_ids = None
        if language is not None:
            lang_ids = [language_to_id(x, gen) for x in langs]
        elif gen.lang_to_id:
            lang_ids = self.detect_language(feats, enc_given if feats is None else None, gen).tolist()
        if lang_ids is not None:
            for i in range(len(rows)):
                rows[i].append(int(lang_ids[i]))
        if task is not None and task not in ("translate", "transcribe"):
            raise ValueError(f"The `{task}` task is not supported. The task should be one of `['translate', 'transcribe']`")
        for r in rows:
            if task is not None:
                r.append(gen.task_to_id[task])
            elif language is not None and gen.task_to_id:
                if not any(t in r for t in gen.task_to_id.values()):
                    r.append(gen.task_to_id["transcribe"])
            if not return_timestamps and r[-1] != gen.no_timestamps_token_id:
                r.append(gen.no_timestamps_token_id)
            elif return_timestamps and r[-1] == gen.no_timestamps_token_id:
                r.pop()
        arr = np.asarray(rows, dtype=np.int64)
        return np.broadcast_to(arr, (B, arr.shape[1])).copy()


def _retrieve_segment(seq, ts_begin, seek_num_frames, time_offset, input_stride=2, time_precision=0.02,
                      time_precision_features=0.01):
    """``_retrieve_segment`` (generation_whisper.py:1977-2074)."""
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
        offset = seek_num_frames if single_ending else (int(seq[last - 2]) - ts_begin) * input_stride
    else:
        stamps = seq[ts]
        last_pos = int(seek_num_frames * time_precision_features / time_precision)
        if stamps.size > 0 and stamps[-1] != ts_begin:
            last_pos = float(stamps[-1] - ts_begin)
        segs = [{"start": time_offset, "end": time_offset + last_pos * time_precision, "tokens": seq}]
        offset = seek_num_frames
    return segs, offset


# HF-style alias
WhisperForConditionalGeneration = KWhisperForConditionalGeneration

"""Shared test helpers (inputs regenerated from seeds; expected values from tests/golden)."""
from __future__ import annotations

import json

import numpy as np

from kwhisper import synthetic as S
from kwhisper.config import PRESETS, generation_constants


def audio_cases(cases):
    out = []
    for c in cases:
        kind, seed = str(c).split(":")
        out.append(getattr(S, f"{kind}_audio")(int(seed)))
    return np.stack(out)


def gen_dict(shape, pad=None) -> dict:
    return generation_constants(shape, pad_token_id=pad).to_dict()


def oracle_features(shape, cases):
    from oracle.mel import log_mel

    return log_mel(audio_cases(cases), shape.num_mel_bins)


def segments_of(fixture_value):
    return json.loads(str(fixture_value))


# mode name -> (generate kwargs, pad override) ; mirrors tools/make_fixtures.py
BASE = dict(language="ja", task="transcribe")
TINY_MODES = {
    "greedy": (dict(BASE, return_timestamps=False), None),
    "greedy_ts": (dict(BASE, return_timestamps=True), None),
    "greedy_dict": (dict(BASE, return_timestamps=False, return_dict_in_generate=True), None),
    "greedy_pad_eq_eos": (dict(BASE, return_timestamps=True), 50257),
    "greedy_translate": (dict(language="ja", task="translate", return_timestamps=False), None),
    "greedy_detect": (dict(return_timestamps=False), None),
    "greedy_short": (dict(BASE, return_timestamps=False, max_length=16), None),
    "beam5": (dict(BASE, return_timestamps=False, num_beams=5, max_length=24), None),
}


# tools/make_fixtures.py BEAM_MODES: name -> (generate kwargs, eos override)
BEAM_MODES = {
    "beam5_ts": (dict(BASE, return_timestamps=True, num_beams=5, max_length=40), None),
    "beam3_eos": (dict(BASE, return_timestamps=False, num_beams=3, max_length=40), 7656),
    "beam4_eos_lp_es": (dict(BASE, return_timestamps=False, num_beams=4, max_length=40, length_penalty=0.5,
                             early_stopping=True), 7656),
    "beam2_eos_never": (dict(BASE, return_timestamps=False, num_beams=2, max_length=40, length_penalty=2.0,
                             early_stopping="never"), 20779),
    "beam3_eos_ts": (dict(BASE, return_timestamps=True, num_beams=3, max_length=40), 7656),
}


def beam_gen_dict(shape, eos=None) -> dict:
    d = gen_dict(shape)
    if eos is not None:
        d["eos_token_id"] = eos
    return d


def long_audio(kind, seed, seconds):
    """tools/make_fixtures.py long_audio: > 30 s clips, the seeded 30 s clips of ``kind`` concatenated."""
    n = int(seconds * 16000)
    parts, k = [], 0
    while sum(len(p) for p in parts) < n:
        parts.append(getattr(S, f"{kind}_audio")(seed + 10 * k))
        k += 1
    return np.concatenate(parts)[:n].astype(np.float32)


def clip_audio(spec):
    """"kind:seed:seconds" -> tools/make_fixtures.py pipeline_audio / long_audio ("reazon": clip ``seed`` of the
    config-4/5 stand-in, kwhisper.synthetic.reazon_audio)."""
    kind, seed, sec = str(spec).split(":")
    if kind == "reazon":
        return S.reazon_audio(int(seed), float(sec))
    return long_audio(kind, int(seed), float(sec))


def longform_inputs(clips, n_mels=80):
    """Batched long-form inputs as the fixture made them -- WhisperFeatureExtractor with truncation=False,
    padding="longest" and the frame-level attention mask (generation_whisper.py:588-589) -- restated by the
    oracle (oracle.mel.log_mel_padded; tokens checked equal to the HF-feature tokens in the build container)."""
    from oracle.mel import log_mel_padded

    audio = [clip_audio(c) for c in clips]
    feats, mask = log_mel_padded(audio, n_mels)
    one, _ = log_mel_padded([audio[1]], n_mels, return_attention_mask=False)
    return feats, mask, one


class OracleFeatureExtractor:
    """The pipeline's feature extractor on the oracle log-mel (test infrastructure): the kwhisper
    WhisperFeatureExtractor's call contract, computed by oracle.mel on the host and moved to the device."""

    sampling_rate, n_samples, padding_value, chunk_length, hop_length = 16000, 480000, 0.0, 30, 160

    def __init__(self, n_mels, device="cuda"):
        import torch

        self.n_mels, self.device = n_mels, torch.device(device)

    def __call__(self, raw_speech, sampling_rate=None, truncation=True, padding="max_length",
                 return_attention_mask=None, **kw):
        import torch
        from oracle.mel import log_mel_padded, pad_or_trim

        clips = [np.asarray(x, dtype=np.float32).reshape(-1) for x in raw_speech]
        if padding != "longest":
            lens = [min(len(c), self.n_samples) for c in clips]
            clips = [pad_or_trim(c) for c in clips]
        feats, mask = log_mel_padded(clips, self.n_mels)
        if padding != "longest":
            mask = np.zeros_like(mask)
            for i, n in enumerate(lens):
                mask[i, : -(-n // self.hop_length)] = 1  # samples 0, 160, ... below n (:333)
        out = {"input_features": torch.from_numpy(feats).to(self.device)}
        if return_attention_mask:
            out["attention_mask"] = torch.from_numpy(mask).to(self.device)
        return out


class StubTok:
    """What the pipeline asks of a Whisper tokenizer (no vocab files offline): ids decode to "[id]" strings,
    a lone special id to "<|name|>".  The fixtures' text was produced by transformers' own _decode_asr over
    this same stub (tools/make_fixtures.py _stub_tokenizer)."""

    def __init__(self, g):
        self.g = g
        self.all_special_ids = list(range(g.eos_token_id, g.no_timestamps_token_id + 1)) + [g.pad_token_id]
        self._names = {g.eos_token_id: "endoftext", g.decoder_start_token_id: "startoftranscript",
                       g.prev_sot_token_id: "startofprev", g.no_timestamps_token_id: "notimestamps",
                       g.task_to_id["translate"]: "translate", g.task_to_id["transcribe"]: "transcribe"}
        for tok, tid in g.lang_to_id.items():
            self._names[tid] = tok[2:-2]

    def convert_tokens_to_ids(self, tok):
        inv = {f"<|{v}|>": k for k, v in self._names.items()}
        return inv[tok]

    def decode(self, ids):
        ids = [int(i) for i in ids]
        if len(ids) == 1 and ids[0] in self._names:
            return f"<|{self._names[ids[0]]}|>"
        return "".join(f"[{i}]" for i in ids)


def jsonable(x):
    """Pipeline results compared through JSON (tuples -> lists), as the fixtures store them."""
    return json.loads(json.dumps(x))

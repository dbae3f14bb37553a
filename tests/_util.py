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


def longform_inputs(clips, n_mels=80):
    """Batched long-form inputs as the fixture made them: transformers' WhisperFeatureExtractor with
    truncation=False, padding="longest" and the frame-level attention mask (generation_whisper.py:588-589)."""
    from transformers import WhisperFeatureExtractor

    fe = WhisperFeatureExtractor(feature_size=n_mels)
    audio = []
    for c in clips:
        kind, seed, sec = str(c).split(":")
        audio.append(long_audio(kind, int(seed), float(sec)))
    inp = fe(audio, sampling_rate=16000, return_tensors="np", truncation=False, padding="longest",
             return_attention_mask=True)
    one = fe([audio[1]], sampling_rate=16000, return_tensors="np", truncation=False, padding="longest")
    return inp["input_features"], inp["attention_mask"], one["input_features"]

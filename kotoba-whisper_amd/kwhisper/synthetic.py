"""Seeded synthetic inputs and weights (no network, no checkpoints offline).

Weights follow the HF ``WhisperForConditionalGeneration`` state-dict naming
(TF/models/whisper/modeling_whisper.py:540-795, :965-1080) so the same dict
loads into the engine and into an HF model.  Every tensor is drawn from its
own numpy PCG64 stream seeded by (seed, crc32(name)), so any tensor can be
regenerated alone, on any host, without transformers.

Audio follows ``run_speed_eval.py:14-17`` (uniform noise of amplitude 0.007
at 16 kHz).
"""
from __future__ import annotations

import math
import zlib

import numpy as np

from .config import WhisperShape


def _rng(seed: int, name: str) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64(np.random.SeedSequence([seed, zlib.crc32(name.encode())])))


def _normal(seed: int, name: str, shape, std: float) -> np.ndarray:
    return _rng(seed, name).standard_normal(shape, dtype=np.float32) * np.float32(std)


def sinusoids(length: int, channels: int, max_timescale: float = 10000.0) -> np.ndarray:
    """``sinusoids`` (modeling_whisper.py:55-64), evaluated in torch-equivalent fp32."""
    log_inc = math.log(max_timescale) / (channels // 2 - 1)
    inv = np.exp(-log_inc * np.arange(channels // 2, dtype=np.float32), dtype=np.float32).astype(np.float32)
    t = np.arange(length, dtype=np.float32)[:, None] * inv[None, :]
    return np.concatenate([np.sin(t), np.cos(t)], axis=1).astype(np.float32)


def state_dict_names(shape: WhisperShape) -> list[tuple[str, tuple]]:
    """(name, shape) of every parameter, in HF state-dict order (proj_out tied, omitted)."""
    d, s = shape.d_model, shape
    out: list[tuple[str, tuple]] = [
        ("model.encoder.conv1.weight", (d, s.num_mel_bins, 3)),
        ("model.encoder.conv1.bias", (d,)),
        ("model.encoder.conv2.weight", (d, d, 3)),
        ("model.encoder.conv2.bias", (d,)),
        ("model.encoder.embed_positions.weight", (s.max_source_positions, d)),
    ]

    def attn(p):
        return [
            (f"{p}.k_proj.weight", (d, d)),
            (f"{p}.v_proj.weight", (d, d)),
            (f"{p}.v_proj.bias", (d,)),
            (f"{p}.q_proj.weight", (d, d)),
            (f"{p}.q_proj.bias", (d,)),
            (f"{p}.out_proj.weight", (d, d)),
            (f"{p}.out_proj.bias", (d,)),
        ]

    def ln(p):
        return [(f"{p}.weight", (d,)), (f"{p}.bias", (d,))]

    for i in range(s.encoder_layers):
        p = f"model.encoder.layers.{i}"
        out += attn(f"{p}.self_attn") + ln(f"{p}.self_attn_layer_norm")
        out += [
            (f"{p}.fc1.weight", (s.encoder_ffn_dim, d)),
            (f"{p}.fc1.bias", (s.encoder_ffn_dim,)),
            (f"{p}.fc2.weight", (d, s.encoder_ffn_dim)),
            (f"{p}.fc2.bias", (d,)),
        ] + ln(f"{p}.final_layer_norm")
    out += ln("model.encoder.layer_norm")
    out += [
        ("model.decoder.embed_tokens.weight", (s.vocab_size, d)),
        ("model.decoder.embed_positions.weight", (s.max_target_positions, d)),
    ]
    for i in range(s.decoder_layers):
        p = f"model.decoder.layers.{i}"
        out += attn(f"{p}.self_attn") + ln(f"{p}.self_attn_layer_norm")
        out += attn(f"{p}.encoder_attn") + ln(f"{p}.encoder_attn_layer_norm")
        out += [
            (f"{p}.fc1.weight", (s.decoder_ffn_dim, d)),
            (f"{p}.fc1.bias", (s.decoder_ffn_dim,)),
            (f"{p}.fc2.weight", (d, s.decoder_ffn_dim)),
            (f"{p}.fc2.bias", (d,)),
        ] + ln(f"{p}.final_layer_norm")
    out += ln("model.decoder.layer_norm")
    return out


def synthetic_tensor(seed: int, name: str, shp: tuple, embed_std: float = 0.1, pos_std: float = 1.0) -> np.ndarray:
    """One parameter of the seeded recipe (fp32)."""
    if name == "model.encoder.embed_positions.weight":
        return sinusoids(*shp)
    if name.endswith("layer_norm.weight"):
        return 1.0 + _normal(seed, name, shp, 0.1)
    if name.endswith(".bias"):
        return _normal(seed, name, shp, 0.1)
    if name == "model.decoder.embed_tokens.weight":
        return _normal(seed, name, shp, embed_std)
    if name == "model.decoder.embed_positions.weight":
        return _normal(seed, name, shp, pos_std)
    fan_in = int(np.prod(shp[1:]))
    return _normal(seed, name, shp, 1.0 / math.sqrt(fan_in))


def synthetic_state_dict(shape: WhisperShape, seed: int = 0, embed_std: float = 0.1, pos_std: float = 1.0) -> dict:
    """Seeded fp32 numpy weights for ``shape`` (HF naming, proj_out tied -> omitted).

    Scales: linear/conv N(0, 1/fan_in); biases N(0, 0.1^2); LayerNorm gamma 1+N(0, 0.1^2);
    token embedding N(0, embed_std^2) (small, so greedy output is not one repeated token);
    decoder positions N(0, pos_std^2); encoder positions = exact sinusoids.
    """
    from concurrent.futures import ThreadPoolExecutor
    import os

    names = state_dict_names(shape)
    # every tensor has its own stream, so drawing them on threads (numpy's generators release the GIL) gives the
    # same values: large-v3's 1.55 B parameters in seconds instead of half a minute
    with ThreadPoolExecutor(max(1, min(16, os.cpu_count() or 1))) as ex:
        vals = list(ex.map(lambda ns: synthetic_tensor(seed, ns[0], ns[1], embed_std, pos_std), names))
    return {n: v for (n, _), v in zip(names, vals)}


def synthetic_state_dict_torch(shape: WhisperShape, seed: int = 0, device="cuda", embed_std: float = 0.1,
                               pos_std: float = 1.0) -> dict:
    """Same recipe and scales as ``synthetic_state_dict`` but drawn with torch's generator on ``device``
    (fast for the 1.5 B-parameter benchmark model; values differ from the numpy recipe)."""
    import torch

    g = torch.Generator(device=device).manual_seed(seed)
    out = {}
    for name, shp in state_dict_names(shape):
        if name == "model.encoder.embed_positions.weight":
            out[name] = torch.from_numpy(sinusoids(*shp)).to(device)
            continue
        t = torch.randn(shp, generator=g, device=device, dtype=torch.float32)
        if name.endswith("layer_norm.weight"):
            t = 1.0 + 0.1 * t
        elif name.endswith(".bias"):
            t *= 0.1
        elif name == "model.decoder.embed_tokens.weight":
            t *= embed_std
        elif name == "model.decoder.embed_positions.weight":
            t *= pos_std
        else:
            t *= 1.0 / math.sqrt(int(np.prod(shp[1:])))
        out[name] = t
    return out


def dummy_audio(seed: int, n_samples: int = 480000) -> np.ndarray:
    """``run_speed_eval.py:14-17``: ``(rand(n) - 0.5) * 2 * 0.007`` with numpy seed ``seed``."""
    rng = np.random.RandomState(seed)
    return ((rng.rand(n_samples) - 0.5) * 2 * 0.007).astype(np.float32)


def tone_audio(seed: int, n_samples: int = 480000, sr: int = 16000) -> np.ndarray:
    """A louder, structured test signal (chirps + noise) for wider log-mel dynamic range."""
    rng = np.random.RandomState(1000 + seed)
    t = np.arange(n_samples, dtype=np.float64) / sr
    f0 = 200.0 + 150.0 * seed
    x = 0.3 * np.sin(2 * np.pi * (f0 * t + 20.0 * t * t)) + 0.05 * rng.randn(n_samples)
    x[: n_samples // 7] *= 0.01  # a quiet head exercises the max-8 clamp
    return x.astype(np.float32)


def reazon_durations(n: int = 1768, seed: int = 0) -> np.ndarray:
    """Clip durations (s) of a synthetic stand-in for the ReazonSpeech "tiny" shard that BASELINE config 4
    pseudo-labels, with the shard's statistics (reference misc/data_statistics.json:1: 1,768 clips, mean
    4.37 s, min 0.62 s, max 21.8 s): gamma-shaped, clipped, rescaled to the mean, extremes present exactly."""
    rng = np.random.default_rng(seed)
    d = rng.gamma(2.2, 4.37 / 2.2, n)
    for _ in range(20):
        d = np.clip(d * (4.37 / d.mean()), 0.62, 21.8)
    d[0], d[1] = 0.62, 21.8
    d *= (4.37 * n - 0.62 - 21.8) / d[2:].sum() if n > 2 else 1.0
    d[0], d[1] = 0.62, 21.8
    return np.clip(d, 0.62, 21.8)


def reazon_audio(i: int, dur: float, sr: int = 16000) -> np.ndarray:
    """Clip ``i`` of the config-4 stand-in: ``run_speed_eval.py:14-17`` noise, ``dur`` seconds (the feature
    extractor zero-pads it to 30 s, feature_extraction_whisper.py:300-307)."""
    rng = np.random.RandomState(1000 + i)
    return ((rng.rand(int(dur * sr)) - 0.5) * 2 * 0.007).astype(np.float32)

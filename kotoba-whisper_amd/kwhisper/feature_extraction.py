"""``WhisperFeatureExtractor`` drop-in whose log-mel runs on the MI355X (kw_log_mel).

Mirrors TF/models/whisper/feature_extraction_whisper.py: constructor fields (:69-103), the slaney
mel filter bank (TF/audio_utils.py:638-743, computed once on the host in float64 exactly as the
reference does), padding/truncation to ``n_samples`` with zeros (:300-307) and the output layout
(B, n_mels, 3000).  The spectrogram itself is the HIP kernel (no CPU fallback).
"""
from __future__ import annotations

import numpy as np
import torch

from . import ops


def _hz_to_mel(f):
    f = np.asarray(f, dtype=np.float64)
    out = 3.0 * f / 200.0
    logstep = 27.0 / np.log(6.4)
    return np.where(f >= 1000.0, 15.0 + np.log(np.maximum(f, 1e-300) / 1000.0) * logstep, out)


def _mel_to_hz(m):
    m = np.asarray(m, dtype=np.float64)
    out = 200.0 * m / 3.0
    return np.where(m >= 15.0, 1000.0 * np.exp(np.log(6.4) / 27.0 * (m - 15.0)), out)


def mel_filter_bank(num_frequency_bins: int, num_mel_filters: int, min_frequency: float, max_frequency: float,
                    sampling_rate: int) -> np.ndarray:
    """Slaney-scale, slaney-normalised triangular filters, shape (num_frequency_bins, num_mel_filters)."""
    mels = np.linspace(_hz_to_mel(min_frequency), _hz_to_mel(max_frequency), num_mel_filters + 2)
    freqs = _mel_to_hz(mels)
    fft_freqs = np.linspace(0, sampling_rate // 2, num_frequency_bins)
    diff = np.diff(freqs)
    slopes = freqs[None, :] - fft_freqs[:, None]
    down = -slopes[:, :-2] / diff[:-1]
    up = slopes[:, 2:] / diff[1:]
    fb = np.maximum(np.zeros(1), np.minimum(down, up))
    fb *= (2.0 / (freqs[2: num_mel_filters + 2] - freqs[:num_mel_filters]))[None, :]
    return fb


class WhisperFeatureExtractor:
    model_input_names = ["input_features"]

    def __init__(self, feature_size=80, sampling_rate=16000, hop_length=160, chunk_length=30, n_fft=400,
                 padding_value=0.0, dither=0.0, return_attention_mask=False, device="cuda", **kwargs):
        if n_fft != 400 or hop_length != 160:
            raise ValueError("the device log-mel kernel implements n_fft=400, hop_length=160 (Whisper)")
        if dither != 0.0:
            raise NotImplementedError("dither != 0 is not supported")
        self.feature_size = feature_size
        self.sampling_rate = sampling_rate
        self.hop_length = hop_length
        self.chunk_length = chunk_length
        self.n_fft = n_fft
        self.padding_value = padding_value
        self.dither = dither
        self.return_attention_mask = return_attention_mask
        self.n_samples = chunk_length * sampling_rate
        self.nb_max_frames = self.n_samples // hop_length
        self.device = torch.device(device)
        self.mel_filters = mel_filter_bank(1 + n_fft // 2, feature_size, 0.0, 8000.0, sampling_rate)
        self._fb_dev = None

    def _filters(self):
        if self._fb_dev is None:
            self._fb_dev = torch.from_numpy(self.mel_filters.astype(np.float32)).to(self.device).contiguous()
        return self._fb_dev

    def extract(self, audio: torch.Tensor) -> torch.Tensor:
        """(B, n_samples) f32 device audio (already padded/truncated) -> (B, n_mels, frames) f32 device."""
        return ops.log_mel(audio, self._filters())

    def __call__(self, raw_speech, sampling_rate=None, return_tensors=None, truncation=True, padding="max_length",
                 max_length=None, return_attention_mask=None, device=None, **kwargs):
        if sampling_rate is not None and sampling_rate != self.sampling_rate:
            raise ValueError(
                f"The model corresponding to this feature extractor: {self.__class__.__name__} was trained using a "
                f"sampling rate of {self.sampling_rate}. Please make sure that the provided `raw_speech` input was "
                f"sampled with {self.sampling_rate} and not {sampling_rate}.")
        if isinstance(raw_speech, torch.Tensor):
            raw_speech = raw_speech.detach().cpu().numpy()
        batched = isinstance(raw_speech, (list, tuple)) and len(raw_speech) > 0 and \
            isinstance(raw_speech[0], (np.ndarray, list, tuple)) or (isinstance(raw_speech, np.ndarray) and raw_speech.ndim > 1)
        if batched and isinstance(raw_speech, np.ndarray) and raw_speech.ndim > 2:
            raise ValueError(f"Only mono-channel audio is supported for input to {self}")
        clips = [np.asarray(x, dtype=np.float32).reshape(-1) for x in raw_speech] if batched else \
            [np.asarray(raw_speech, dtype=np.float32).reshape(-1)]
        n = max_length or self.n_samples
        if padding == "longest":
            n = max(len(c) for c in clips)
            n = -(-n // self.hop_length) * self.hop_length
        buf = np.full((len(clips), n), self.padding_value, dtype=np.float32)
        mask = np.zeros((len(clips), n), dtype=np.int32)
        for i, c in enumerate(clips):
            c = c[:n] if truncation else c
            buf[i, : len(c)] = c
            mask[i, : len(c)] = 1
        audio = torch.from_numpy(buf).to(self.device)
        feats = self.extract(audio)
        out = {"input_features": feats}
        if return_attention_mask or (return_attention_mask is None and self.return_attention_mask):
            out["attention_mask"] = torch.from_numpy(mask[:, :: self.hop_length][:, : feats.shape[-1]]).to(self.device)
        if return_tensors == "np":
            out = {k: v.cpu().numpy() for k, v in out.items()}
        return out

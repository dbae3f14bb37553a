"""Oracle log-mel (TEST INFRASTRUCTURE ONLY -- see oracle/__init__.py).

Restates, in numpy:
  * ``mel_filter_bank(norm="slaney", mel_scale="slaney")``  TF/audio_utils.py:638-743
    (hertz_to_mel :448-480, mel_to_hertz :483-518, triangles :541-560);
  * ``WhisperFeatureExtractor._torch_extract_fbank_features``
    TF/models/whisper/feature_extraction_whisper.py:135-168, i.e.
    ``torch.stft(n_fft=400, hop=160, hann(periodic), center=True, pad_mode="reflect")``,
    ``|X|^2``, drop the last frame, ``mel_filters.T @ P``, ``log10(clamp(1e-10))``,
    per-clip ``max(x, max-8)``, ``(x+4)/4``;
  * padding/truncation to 480,000 samples (``__call__`` :300-307, zero padding).
"""
from __future__ import annotations

import numpy as np

N_FFT = 400
HOP = 160
N_SAMPLES = 480000
N_FRAMES = 3000


def _hz_to_mel_slaney(f):
    f = np.asarray(f, dtype=np.float64)
    mel = 3.0 * f / 200.0
    log_region = f >= 1000.0
    mel = np.where(log_region, 15.0 + np.log(np.maximum(f, 1e-30) / 1000.0) * (27.0 / np.log(6.4)), mel)
    return mel


def _mel_to_hz_slaney(m):
    m = np.asarray(m, dtype=np.float64)
    f = 200.0 * m / 3.0
    return np.where(m >= 15.0, 1000.0 * np.exp((np.log(6.4) / 27.0) * (m - 15.0)), f)


def mel_filters(n_mels: int, sr: int = 16000, n_fft: int = N_FFT) -> np.ndarray:
    """(n_fft//2+1, n_mels) float64 slaney filter bank, 0..8 kHz."""
    n_bins = n_fft // 2 + 1
    mels = np.linspace(_hz_to_mel_slaney(0.0), _hz_to_mel_slaney(8000.0), n_mels + 2)
    centers = _mel_to_hz_slaney(mels)
    fft_freqs = np.linspace(0, sr // 2, n_bins)
    diff = np.diff(centers)
    slopes = centers[None, :] - fft_freqs[:, None]
    down = -slopes[:, :-2] / diff[:-1]
    up = slopes[:, 2:] / diff[1:]
    fb = np.maximum(0.0, np.minimum(down, up))
    fb *= (2.0 / (centers[2 : n_mels + 2] - centers[:n_mels]))[None, :]
    return fb


def pad_or_trim(audio: np.ndarray, n: int = N_SAMPLES) -> np.ndarray:
    a = np.asarray(audio, dtype=np.float32).reshape(-1)[:n]
    return np.pad(a, (0, n - a.shape[0])) if a.shape[0] < n else a


def log_mel(audio_batch: np.ndarray, n_mels: int) -> np.ndarray:
    """(B, 480000) f32 audio -> (B, n_mels, 3000) f32 log-mel, reference arithmetic in f32/f64.

    The STFT is evaluated with numpy's FFT in float64 and rounded to f32 power,
    i.e. a more exact evaluation of the same algorithm; the reference's own docstring
    quotes 1e-5 agreement between its numpy and torch paths (feature_extraction_whisper.py:107).
    """
    x = np.asarray(audio_batch, dtype=np.float32)
    if x.ndim == 1:
        x = x[None]
    b, n = x.shape
    window = (0.5 - 0.5 * np.cos(2.0 * np.pi * np.arange(N_FFT) / N_FFT)).astype(np.float32)
    pad = N_FFT // 2
    xp = np.pad(x, ((0, 0), (pad, pad)), mode="reflect")
    n_frames = 1 + (xp.shape[1] - N_FFT) // HOP
    idx = np.arange(N_FFT)[None, :] + HOP * np.arange(n_frames)[:, None]
    fb = mel_filters(n_mels).astype(np.float32)
    out = np.empty((b, n_mels, n_frames - 1), dtype=np.float32)
    for i in range(b):
        frames = xp[i][idx].astype(np.float64) * window.astype(np.float64)
        spec = np.fft.rfft(frames, axis=1)
        power = (spec.real ** 2 + spec.imag ** 2).astype(np.float32)[:-1]  # drop last frame
        mel = (fb.T.astype(np.float64) @ power.T.astype(np.float64)).astype(np.float32)
        lg = np.log10(np.maximum(mel, np.float32(1e-10)))
        lg = np.maximum(lg, lg.max() - np.float32(8.0))
        out[i] = (lg + np.float32(4.0)) / np.float32(4.0)
    return out


def log_mel_padded(audio_list, n_mels: int, return_attention_mask: bool = True):
    """``WhisperFeatureExtractor.__call__(raw, padding="longest", truncation=False,
    return_attention_mask=True)`` (TF/models/whisper/feature_extraction_whisper.py:280-346): every clip is
    zero-padded to the longest clip of the batch (``SequenceFeatureExtractor.pad``), the log-mel runs over
    that length (per-clip max clamp over the padded clip), and the sample-level mask is subsampled by the
    hop (``[:, ::160]``, minus the last entry when the length is not a multiple of 160, :333-340).

    Returns (features (B, n_mels, L // 160) f32, attention_mask (B, L // 160) int32 or None)."""
    clips = [np.asarray(a, dtype=np.float32).reshape(-1) for a in audio_list]
    n = max(c.shape[0] for c in clips)
    batch = np.zeros((len(clips), n), dtype=np.float32)
    mask = np.zeros((len(clips), n), dtype=np.int32)
    for i, c in enumerate(clips):
        batch[i, : c.shape[0]] = c
        mask[i, : c.shape[0]] = 1
    feats = log_mel(batch, n_mels)
    if not return_attention_mask:
        return feats, None
    m = mask[:, ::HOP]
    if n % HOP != 0:
        m = m[:, :-1]
    return feats, m

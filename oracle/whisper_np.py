"""Oracle Whisper forward in numpy fp32 (TEST INFRASTRUCTURE ONLY -- see oracle/__init__.py).

Restates TF/models/whisper/modeling_whisper.py (transformers 5.15.0):
  * encoder  :592-646  -- gelu(conv1), gelu(conv2) (k3, p1, stride 1/2), +embed_positions,
    pre-LN layers :379-413, final LayerNorm :642;
  * attention :284-356 -- q = (x Wq + bq) * head_dim**-0.5 *before* QK^T (:309), k without
    bias (:279), softmax(QK^T) V with scale 1.0 (sdpa_attention.py:79-166), causal only for
    decoder self-attention with q_len > 1 (sdpa_attention.py:120);
  * decoder :690-795 -- embed_tokens + embed_positions[past_len:past_len+q] (:737-762, no
    embed scale), layers :448-505 (self, cross, FFN), final LayerNorm :790;
  * proj_out tied to embed_tokens (:965,1080), logits cast to f32 (TF/generation/utils.py:2894).
GELU is the exact erf form (TF/activations.py:70-89), LayerNorm eps 1e-5.
"""
from __future__ import annotations

import numpy as np
from scipy.special import erf


def _gelu(x: np.ndarray) -> np.ndarray:
    return (0.5 * x * (1.0 + erf(x / np.float32(np.sqrt(2.0))))).astype(np.float32)


def _ln(x: np.ndarray, w: np.ndarray, b: np.ndarray, eps: float = 1e-5) -> np.ndarray:
    mu = x.mean(-1, keepdims=True, dtype=np.float64)
    var = ((x - mu) ** 2).mean(-1, keepdims=True, dtype=np.float64)
    return (((x - mu) / np.sqrt(var + eps)) * w + b).astype(np.float32)


def _softmax(x: np.ndarray) -> np.ndarray:
    m = x.max(-1, keepdims=True)
    e = np.exp(x - m)
    return (e / e.sum(-1, keepdims=True)).astype(np.float32)


class WhisperNP:
    """Numpy fp32 Whisper with an explicit (growing) KV cache."""

    def __init__(self, sd: dict, shape):
        self.sd = {k: np.asarray(v, dtype=np.float32) for k, v in sd.items()}
        self.s = shape
        self.h = shape.encoder_attention_heads
        self.hd = shape.d_model // self.h

    def _w(self, name):
        return self.sd[name]

    def _lin(self, x, p, bias=True):
        y = x @ self._w(p + ".weight").T
        if bias:
            y = y + self._w(p + ".bias")
        return y.astype(np.float32)

    def _conv(self, x, p, stride):
        # x (B, C, T); Conv1d(k=3, padding=1, stride)
        w, b = self._w(p + ".weight"), self._w(p + ".bias")
        xp = np.pad(x, ((0, 0), (0, 0), (1, 1)))
        t_out = (x.shape[2] + 2 - 3) // stride + 1
        y = np.zeros((x.shape[0], w.shape[0], t_out), dtype=np.float32)
        for k in range(3):
            seg = xp[:, :, k : k + stride * (t_out - 1) + 1 : stride]  # (B, C, T_out)
            y += np.einsum("oc,bct->bot", w[:, :, k], seg, optimize=True).astype(np.float32)
        return (y + b[None, :, None]).astype(np.float32)

    def _heads(self, x):
        b, t, _ = x.shape
        return x.reshape(b, t, self.h, self.hd).transpose(0, 2, 1, 3)

    def _attend(self, q, k, v, causal_offset=None):
        s = q @ k.transpose(0, 1, 3, 2)
        if causal_offset is not None and q.shape[2] > 1:
            tq, tk = q.shape[2], k.shape[2]
            mask = np.arange(tk)[None, :] > (np.arange(tq)[:, None] + causal_offset)
            s = np.where(mask, np.float32(-np.inf), s)
        p = _softmax(s.astype(np.float32))
        o = p @ v
        b, h, t, hd = o.shape
        return o.transpose(0, 2, 1, 3).reshape(b, t, h * hd).astype(np.float32)

    # ---- encoder -------------------------------------------------------------------------
    def encode(self, mel: np.ndarray) -> np.ndarray:
        mel = np.asarray(mel, dtype=np.float32)
        if mel.shape[-1] != self.s.n_frames:
            raise ValueError(
                f"Whisper expects the mel input features to be of length {self.s.n_frames}, "
                f"but found {mel.shape[-1]}."
            )
        x = _gelu(self._conv(mel, "model.encoder.conv1", 1))
        x = _gelu(self._conv(x, "model.encoder.conv2", 2))
        x = x.transpose(0, 2, 1) + self._w("model.encoder.embed_positions.weight")[None]
        x = x.astype(np.float32)
        for i in range(self.s.encoder_layers):
            p = f"model.encoder.layers.{i}"
            h = _ln(x, self._w(p + ".self_attn_layer_norm.weight"), self._w(p + ".self_attn_layer_norm.bias"))
            q = self._heads(self._lin(h, p + ".self_attn.q_proj") * np.float32(self.hd ** -0.5))
            k = self._heads(self._lin(h, p + ".self_attn.k_proj", bias=False))
            v = self._heads(self._lin(h, p + ".self_attn.v_proj"))
            x = x + self._lin(self._attend(q, k, v), p + ".self_attn.out_proj")
            h = _ln(x, self._w(p + ".final_layer_norm.weight"), self._w(p + ".final_layer_norm.bias"))
            x = (x + self._lin(_gelu(self._lin(h, p + ".fc1")), p + ".fc2")).astype(np.float32)
        return _ln(x, self._w("model.encoder.layer_norm.weight"), self._w("model.encoder.layer_norm.bias"))

    # ---- decoder -------------------------------------------------------------------------
    def new_cache(self, enc: np.ndarray) -> dict:
        """Cross K/V computed once (modeling_whisper.py:323-335); self K/V grow per step."""
        cross = []
        for i in range(self.s.decoder_layers):
            p = f"model.decoder.layers.{i}.encoder_attn"
            cross.append((self._heads(self._lin(enc, p + ".k_proj", bias=False)), self._heads(self._lin(enc, p + ".v_proj"))))
        return {"cross": cross, "self": [None] * self.s.decoder_layers, "len": 0}

    def decode(self, ids: np.ndarray, cache: dict) -> np.ndarray:
        """ids (B, q) int -> logits (B, q, V) f32; appends q positions to the cache."""
        ids = np.asarray(ids, dtype=np.int64)
        past = cache["len"]
        q_len = ids.shape[1]
        if past + q_len > self.s.max_target_positions:
            raise ValueError("decoder position overflow")
        x = self._w("model.decoder.embed_tokens.weight")[ids] + self._w("model.decoder.embed_positions.weight")[past : past + q_len][None]
        x = x.astype(np.float32)
        for i in range(self.s.decoder_layers):
            p = f"model.decoder.layers.{i}"
            h = _ln(x, self._w(p + ".self_attn_layer_norm.weight"), self._w(p + ".self_attn_layer_norm.bias"))
            q = self._heads(self._lin(h, p + ".self_attn.q_proj") * np.float32(self.hd ** -0.5))
            k = self._heads(self._lin(h, p + ".self_attn.k_proj", bias=False))
            v = self._heads(self._lin(h, p + ".self_attn.v_proj"))
            if cache["self"][i] is not None:
                k = np.concatenate([cache["self"][i][0], k], axis=2)
                v = np.concatenate([cache["self"][i][1], v], axis=2)
            cache["self"][i] = (k, v)
            x = x + self._lin(self._attend(q, k, v, causal_offset=past), p + ".self_attn.out_proj")
            h = _ln(x, self._w(p + ".encoder_attn_layer_norm.weight"), self._w(p + ".encoder_attn_layer_norm.bias"))
            q = self._heads(self._lin(h, p + ".encoder_attn.q_proj") * np.float32(self.hd ** -0.5))
            ck, cv = cache["cross"][i]
            x = x + self._lin(self._attend(q, ck, cv), p + ".encoder_attn.out_proj")
            h = _ln(x, self._w(p + ".final_layer_norm.weight"), self._w(p + ".final_layer_norm.bias"))
            x = (x + self._lin(_gelu(self._lin(h, p + ".fc1")), p + ".fc2")).astype(np.float32)
        cache["len"] = past + q_len
        x = _ln(x, self._w("model.decoder.layer_norm.weight"), self._w("model.decoder.layer_norm.bias"))
        return (x @ self._w("model.decoder.embed_tokens.weight").T).astype(np.float32)

    @staticmethod
    def reorder(cache: dict, idx: np.ndarray) -> None:
        """Beam reorder of the self cache (cache_utils.py:2035-2038); cross K/V are per item here."""
        cache["self"] = [(k[idx], v[idx]) if k is not None else None for (k, v) in
                         [(c if c is not None else (None, None)) for c in cache["self"]]]

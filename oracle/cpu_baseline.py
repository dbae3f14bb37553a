"""CPU baseline for bench.py -- TEST/MEASUREMENT INFRASTRUCTURE ONLY (see oracle/__init__.py).

Times the reference's own hot path on the host cores: transformers 5.15.0
``WhisperForConditionalGeneration.generate`` in fp32 on CPU (what kotoba-whisper runs at
run_pseudo_labelling.py:338 when no GPU is present; run_speed_eval.py:53-59 uses fp32 on CPU), with
random weights of the named architecture, ``language="ja", task="transcribe"``, greedy, the same
max_length.  Timed like run_speed_eval.py:73-78 (warm-up excluded).

Threads (``torch.set_num_threads(os.cpu_count())``): every CPU this process may use --
``len(os.sched_getaffinity(0))`` -- capped by ``OMP_NUM_THREADS`` when the host sets it.  The GPU box's
harness sets it to 16, the host-CPU share of one GPU (the node's 256 CPUs serve 8 GPUs' jobs); the count
used and the node's CPUs are both reported.
"""
from __future__ import annotations

import os
import time

import torch


def cpu_share() -> int:
    """CPUs this process may use (affinity), capped by OMP_NUM_THREADS if set."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def hf_cpu_generate_rate(shape, batch: int, max_length: int, threads: int | None = None, seed: int = 0) -> dict:
    from transformers import GenerationConfig, WhisperConfig, WhisperForConditionalGeneration
    from transformers.utils import logging as hf_logging

    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "kotoba-whisper_amd"))
    from kwhisper.config import generation_constants
    from kwhisper.synthetic import dummy_audio

    hf_logging.set_verbosity_error()
    threads = threads or cpu_share()
    torch.set_num_threads(threads)
    cfg = WhisperConfig(
        vocab_size=shape.vocab_size, num_mel_bins=shape.num_mel_bins, d_model=shape.d_model,
        encoder_layers=shape.encoder_layers, encoder_attention_heads=shape.encoder_attention_heads,
        encoder_ffn_dim=shape.encoder_ffn_dim, decoder_layers=shape.decoder_layers,
        decoder_attention_heads=shape.decoder_attention_heads, decoder_ffn_dim=shape.decoder_ffn_dim,
        decoder_start_token_id=50258, pad_token_id=50256, eos_token_id=50257, bos_token_id=50257)
    with torch.device("meta"):
        m = WhisperForConditionalGeneration(cfg)
    m = m.to_empty(device="cpu").eval()
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if p.dim() >= 2:
                p.normal_(0.0, 1.0 / (p[0].numel() ** 0.5), generator=g)
            elif "layer_norm.weight" in n:
                p.fill_(1.0)
            else:
                p.normal_(0.0, 0.1, generator=g)
        m.model.decoder.embed_tokens.weight.mul_(0.1)
    m.tie_weights()
    gc = generation_constants(shape)
    m.generation_config = GenerationConfig(**{k: v for k, v in gc.to_dict().items() if k not in ("language", "task")})
    from transformers import WhisperFeatureExtractor

    fe = WhisperFeatureExtractor(feature_size=shape.num_mel_bins)
    feats = torch.from_numpy(fe([dummy_audio(s) for s in range(batch)], sampling_rate=16000,
                                return_tensors="np")["input_features"])
    with torch.no_grad():
        m.generate(feats[:1], max_length=4, language="ja", task="transcribe")  # warm-up
        t0 = time.perf_counter()
        out = m.generate(feats, max_length=max_length, language="ja", task="transcribe")
        dt = time.perf_counter() - t0
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = None
    return {"seconds": dt, "batch": batch, "new_tokens": int(out.shape[1]), "threads": threads,
            "nproc": os.cpu_count(), "affinity_cpus": affinity, "audio_seconds_per_second": batch * 30.0 / dt}

"""kwhisper -- MI355X-native (gfx950) Whisper teacher hot path behind the HF generate() API.

The compute is the HIP library ``libkwhisper.so`` (C ABI: include/kwhisper.h); this package is the
host side that mirrors the reference's Python interface (transformers 5.15.0
``WhisperForConditionalGeneration.generate`` / ``WhisperFeatureExtractor`` as called by
kotoba-whisper's run_pseudo_labelling.py:338).
"""
from .config import KOTOBA_V2, LARGE_V3, PRESETS, TINY, GenerationConstants, WhisperShape, generation_constants

__all__ = [
    "KOTOBA_V2", "LARGE_V3", "PRESETS", "TINY", "GenerationConstants", "WhisperShape", "generation_constants",
    "WhisperEngine", "KWhisperForConditionalGeneration", "WhisperForConditionalGeneration", "WhisperFeatureExtractor",
]


def __getattr__(name):
    if name == "WhisperEngine":
        from .engine import WhisperEngine

        return WhisperEngine
    if name in ("KWhisperForConditionalGeneration", "WhisperForConditionalGeneration"):
        from . import generation

        return getattr(generation, name)
    if name == "WhisperFeatureExtractor":
        from .feature_extraction import WhisperFeatureExtractor

        return WhisperFeatureExtractor
    raise AttributeError(name)

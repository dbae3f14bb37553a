"""Model shapes and generation constants for the Whisper teacher path.

Mirrors the fields of ``transformers.WhisperConfig`` that the hot path reads
(TF/models/whisper/configuration_whisper.py) and the Whisper generation
constants that ``WhisperGenerationMixin.generate`` reads from
``generation_config`` (TF/models/whisper/generation_whisper.py:1455-1608,
1774-1812, 1920-1946).  ``TF/`` = transformers 5.15.0 site-packages.

The public ``generation_config.json`` files of openai/whisper-* are not in
this container; the presets below restate their layout (SURVEY.md §8c
"Constants").  Parity never depends on them: the oracle and the engine are
handed the same ``GenerationConstants`` object.
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field

# TF/models/whisper/tokenization_whisper.py LANGUAGES (order defines token ids).
LANGUAGES = [
    ("en", "english"), ("zh", "chinese"), ("de", "german"), ("es", "spanish"), ("ru", "russian"),
    ("ko", "korean"), ("fr", "french"), ("ja", "japanese"), ("pt", "portuguese"), ("tr", "turkish"),
    ("pl", "polish"), ("ca", "catalan"), ("nl", "dutch"), ("ar", "arabic"), ("sv", "swedish"),
    ("it", "italian"), ("id", "indonesian"), ("hi", "hindi"), ("fi", "finnish"), ("vi", "vietnamese"),
    ("he", "hebrew"), ("uk", "ukrainian"), ("el", "greek"), ("ms", "malay"), ("cs", "czech"),
    ("ro", "romanian"), ("da", "danish"), ("hu", "hungarian"), ("ta", "tamil"), ("no", "norwegian"),
    ("th", "thai"), ("ur", "urdu"), ("hr", "croatian"), ("bg", "bulgarian"), ("lt", "lithuanian"),
    ("la", "latin"), ("mi", "maori"), ("ml", "malayalam"), ("cy", "welsh"), ("sk", "slovak"),
    ("te", "telugu"), ("fa", "persian"), ("lv", "latvian"), ("bn", "bengali"), ("sr", "serbian"),
    ("az", "azerbaijani"), ("sl", "slovenian"), ("kn", "kannada"), ("et", "estonian"), ("mk", "macedonian"),
    ("br", "breton"), ("eu", "basque"), ("is", "icelandic"), ("hy", "armenian"), ("ne", "nepali"),
    ("mn", "mongolian"), ("bs", "bosnian"), ("kk", "kazakh"), ("sq", "albanian"), ("sw", "swahili"),
    ("gl", "galician"), ("mr", "marathi"), ("pa", "punjabi"), ("si", "sinhala"), ("km", "khmer"),
    ("sn", "shona"), ("yo", "yoruba"), ("so", "somali"), ("af", "afrikaans"), ("oc", "occitan"),
    ("ka", "georgian"), ("be", "belarusian"), ("tg", "tajik"), ("sd", "sindhi"), ("gu", "gujarati"),
    ("am", "amharic"), ("yi", "yiddish"), ("lo", "lao"), ("uz", "uzbek"), ("fo", "faroese"),
    ("ht", "haitian creole"), ("ps", "pashto"), ("tk", "turkmen"), ("nn", "nynorsk"), ("mt", "maltese"),
    ("sa", "sanskrit"), ("lb", "luxembourgish"), ("my", "myanmar"), ("bo", "tibetan"), ("tl", "tagalog"),
    ("mg", "malagasy"), ("as", "assamese"), ("tt", "tatar"), ("haw", "hawaiian"), ("ln", "lingala"),
    ("ha", "hausa"), ("ba", "bashkir"), ("jw", "javanese"), ("su", "sundanese"), ("yue", "cantonese"),
]
TASK_IDS = ["translate", "transcribe"]

# Whisper's suppress list (v1/v2 vocabulary, 51865).  The last five entries are
# special tokens and shift by +1 in the v3 vocabulary (one extra language).
_SUPPRESS_TEXT = [
    1, 2, 7, 8, 9, 10, 14, 25, 26, 27, 28, 29, 31, 58, 59, 60, 61, 62, 63, 90, 91, 92, 93, 359, 503, 522,
    542, 873, 893, 902, 918, 922, 931, 1350, 1853, 1982, 2460, 2627, 3246, 3253, 3268, 3536, 3846, 3961,
    4183, 4667, 6585, 6647, 7273, 9061, 9383, 10428, 10929, 11938, 12033, 12331, 12562, 13793, 14157,
    14635, 15265, 15618, 16553, 16604, 18362, 18956, 20075, 21675, 22520, 26130, 26161, 26435, 28279,
    29464, 31650, 32302, 32470, 36865, 42863, 47425, 49870, 50254, 50258,
]


@dataclass(frozen=True)
class WhisperShape:
    """The ``WhisperConfig`` fields the hot path depends on."""

    name: str
    vocab_size: int
    num_mel_bins: int
    d_model: int
    encoder_layers: int
    encoder_attention_heads: int
    encoder_ffn_dim: int
    decoder_layers: int
    decoder_attention_heads: int
    decoder_ffn_dim: int
    max_source_positions: int = 1500
    max_target_positions: int = 448
    decoder_start_token_id: int = 50258
    pad_token_id: int = 50256
    eos_token_id: int = 50257
    bos_token_id: int = 50257
    layer_norm_eps: float = 1e-5

    @property
    def head_dim(self) -> int:
        return self.d_model // self.encoder_attention_heads

    @property
    def n_frames(self) -> int:
        # conv1 stride 1 * conv2 stride 2 * max_source_positions (modeling_whisper.py:612)
        return 2 * self.max_source_positions

    @property
    def is_v3_vocab(self) -> bool:
        return self.vocab_size >= 51866

    def param_count(self) -> int:
        """Parameter count of WhisperForConditionalGeneration (tied proj_out)."""
        d, dm = self.d_model, self.num_mel_bins
        enc = dm * d * 3 + d + d * d * 3 + d + self.max_source_positions * d
        attn = 4 * d * d + 3 * d  # q,v,o bias; k no bias
        enc_layer = attn + 2 * d + d * self.encoder_ffn_dim * 2 + self.encoder_ffn_dim + d + 2 * d
        enc += self.encoder_layers * enc_layer + 2 * d
        dec = self.vocab_size * d + self.max_target_positions * d
        dec_layer = 2 * attn + 2 * d * 2 + d * self.decoder_ffn_dim * 2 + self.decoder_ffn_dim + d + 2 * d
        dec += self.decoder_layers * dec_layer + 2 * d
        return enc + dec


TINY = WhisperShape("openai/whisper-tiny", 51865, 80, 384, 4, 6, 1536, 4, 6, 1536)
LARGE_V3 = WhisperShape("openai/whisper-large-v3", 51866, 128, 1280, 32, 20, 5120, 32, 20, 5120)
KOTOBA_V2 = WhisperShape("kotoba-tech/kotoba-whisper-v2.0", 51866, 128, 1280, 32, 20, 5120, 2, 20, 5120)
PRESETS = {s.name: s for s in (TINY, LARGE_V3, KOTOBA_V2)}
PRESETS.update({"tiny": TINY, "large-v3": LARGE_V3, "kotoba-v2.0": KOTOBA_V2})


@dataclass
class GenerationConstants:
    """Generation-config fields read by the Whisper generate path.

    Field names follow ``transformers.GenerationConfig`` so that the same
    object can be handed to both the engine and an HF model.
    """

    decoder_start_token_id: int
    eos_token_id: int
    pad_token_id: int
    bos_token_id: int
    no_timestamps_token_id: int
    prev_sot_token_id: int
    suppress_tokens: list
    begin_suppress_tokens: list
    lang_to_id: dict
    task_to_id: dict
    max_initial_timestamp_index: int = 50
    max_length: int = 448
    is_multilingual: bool = True
    return_timestamps: bool = False
    num_beams: int = 1
    length_penalty: float = 1.0
    early_stopping: bool = False
    language: str | None = None
    task: str | None = None
    forced_decoder_ids: list | None = None

    @property
    def timestamp_begin(self) -> int:
        return self.no_timestamps_token_id + 1

    def copy(self) -> "GenerationConstants":
        return dataclasses.replace(
            self,
            suppress_tokens=list(self.suppress_tokens) if self.suppress_tokens is not None else None,
            begin_suppress_tokens=list(self.begin_suppress_tokens) if self.begin_suppress_tokens is not None else None,
            lang_to_id=dict(self.lang_to_id),
            task_to_id=dict(self.task_to_id),
        )

    def to_dict(self) -> dict:
        return dataclasses.asdict(self)


def generation_constants(shape: WhisperShape, pad_token_id: int | None = None) -> GenerationConstants:
    """The multilingual Whisper generation constants for ``shape``'s vocabulary."""
    n_lang = 100 if shape.is_v3_vocab else 99
    langs = LANGUAGES[:n_lang]
    first_lang = 50259
    lang_to_id = {f"<|{code}|>": first_lang + i for i, (code, _) in enumerate(langs)}
    after = first_lang + n_lang  # translate
    translate, transcribe = after, after + 1
    prev_sot = after + 3
    no_ts = after + 5
    suppress = _SUPPRESS_TEXT + [after, after + 1, after + 2, after + 3, after + 4]
    return GenerationConstants(
        decoder_start_token_id=shape.decoder_start_token_id,
        eos_token_id=shape.eos_token_id,
        pad_token_id=shape.pad_token_id if pad_token_id is None else pad_token_id,
        bos_token_id=shape.bos_token_id,
        no_timestamps_token_id=no_ts,
        prev_sot_token_id=prev_sot,
        suppress_tokens=suppress,
        begin_suppress_tokens=[220, shape.eos_token_id],
        lang_to_id=lang_to_id,
        task_to_id={"translate": translate, "transcribe": transcribe},
    )


def language_to_id(language: str, gen: GenerationConstants) -> int:
    """``_retrieve_init_tokens.language_to_id`` (generation_whisper.py:1464-1485)."""
    lang = language.lower()
    codes = {code: name for code, name in LANGUAGES}
    names = {name: code for code, name in LANGUAGES}
    if lang in gen.lang_to_id:
        tok = lang
    elif lang in names:
        tok = f"<|{names[lang]}|>"
    elif lang in codes:
        tok = f"<|{lang}|>"
    else:
        is_code = len(lang) == 2
        raise ValueError(
            f"Unsupported language: {lang}. Language should be one of:"
            f" {list(codes.keys()) if is_code else list(names.keys())}."
        )
    if tok not in gen.lang_to_id:
        raise ValueError(
            f"{tok} is not supported by this specific model as it is not in the `generation_config.lang_to_id`."
            " (You should just add it to the generation config)"
        )
    return gen.lang_to_id[tok]

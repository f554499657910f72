"""Model dimensions, special-token layout and generation settings of the Whisper hot path.

The reference never states these itself: it names a hub checkpoint
(`openai/whisper-large-v3`, /root/reference/vocalis/core/audio_pipeline.py:171) and lets
transformers resolve `config.json` / `generation_config.json`. Real checkpoints are not on disk
here, so the values are restated from the public Whisper model cards (dims) and from transformers'
Whisper generation logic ($TF/models/whisper/generation_whisper.py). When a local checkpoint
directory is given, `GenerationSettings.from_checkpoint` reads its own generation_config.json.
"""
from __future__ import annotations

import dataclasses
import json
import os
from typing import Dict, List, Optional, Tuple

# Whisper language codes in token order (<|en|> = first language token). 99 for v1/v2 vocabularies,
# the v3 vocabulary (51866) adds "yue" as the 100th.
LANGUAGE_CODES: List[str] = (
    "en zh de es ru ko fr ja pt tr pl ca nl ar sv it id hi fi vi he uk el ms cs ro da hu ta no th ur hr bg "
    "lt la mi ml cy sk te fa lv bn sr az sl kn et mk br eu is hy ne mn bs kk sq sw gl mr pa si km sn yo so "
    "af oc ka be tg sd gu am yi lo uz fo ht ps tk nn mt sa lb my bo tl mg as tt haw ln ha ba jw su yue"
).split()


@dataclasses.dataclass(frozen=True)
class WhisperDims:
    """Architecture hyper-parameters (WhisperConfig fields)."""

    name: str
    d_model: int
    encoder_layers: int
    decoder_layers: int
    heads: int
    ffn: int
    n_mels: int
    vocab: int
    max_source_positions: int = 1500
    max_target_positions: int = 448

    @property
    def head_dim(self) -> int:
        return self.d_model // self.heads

    def validate(self) -> None:
        if self.d_model % 64 or self.head_dim != 64:
            raise ValueError(f"{self.name}: head_dim must be 64 (d_model={self.d_model}, heads={self.heads})")
        if self.ffn % 128 or self.d_model % 128:
            raise ValueError(f"{self.name}: d_model/ffn must be multiples of 128")


PRESETS: Dict[str, WhisperDims] = {
    # BASELINE.json configs[1..4]: openai/whisper-large-v3-turbo
    "large-v3-turbo": WhisperDims("large-v3-turbo", 1280, 32, 4, 20, 5120, 128, 51866),
    # reference default model name (audio_pipeline.py:171)
    "large-v3": WhisperDims("large-v3", 1280, 32, 32, 20, 5120, 128, 51866),
    # BASELINE.json configs[0]: whisper-tiny.en (English-only vocabulary)
    "tiny.en": WhisperDims("tiny.en", 384, 4, 4, 6, 1536, 80, 51864),
    "tiny": WhisperDims("tiny", 384, 4, 4, 6, 1536, 80, 51865),
    "base": WhisperDims("base", 512, 6, 6, 8, 2048, 80, 51865),
    # small synthetic config used by the parity tests (multilingual v3 vocabulary, 128 mels)
    "test-mini": WhisperDims("test-mini", 256, 2, 2, 4, 1024, 128, 51866),
}


@dataclasses.dataclass(frozen=True)
class SpecialTokens:
    """Token-id layout of a Whisper vocabulary (derived from its size, as the checkpoints lay it out)."""

    vocab: int
    eot: int
    sot: int
    lang_begin: int
    n_languages: int
    translate: int
    transcribe: int
    startoflm: int
    startofprev: int
    nospeech: int
    notimestamps: int
    is_multilingual: bool

    @property
    def timestamp_begin(self) -> int:
        return self.notimestamps + 1

    @property
    def lang_end(self) -> int:
        return self.lang_begin + self.n_languages

    def lang_to_id(self) -> Dict[str, int]:
        return {f"<|{c}|>": self.lang_begin + i for i, c in enumerate(LANGUAGE_CODES[: self.n_languages])}

    def special_ids(self) -> List[int]:
        """ids the tokenizer reports in all_special_ids (everything between eot and the timestamps)."""
        return list(range(self.eot, self.timestamp_begin))

    @staticmethod
    def for_vocab(vocab: int) -> "SpecialTokens":
        if vocab == 51866:  # v3: 100 languages
            n_lang, eot, multi = 100, 50257, True
        elif vocab == 51865:  # v1/v2 multilingual: 99 languages
            n_lang, eot, multi = 99, 50257, True
        elif vocab == 51864:  # English-only (.en): same 99 language tokens, never prompted
            n_lang, eot, multi = 99, 50256, False
        else:
            raise ValueError(f"unsupported Whisper vocabulary size {vocab}")
        sot = eot + 1
        lb = sot + 1
        translate = lb + n_lang
        transcribe = translate + 1
        startoflm = transcribe + 1
        startofprev = startoflm + 1
        nospeech = startofprev + 1
        notimestamps = nospeech + 1
        st = SpecialTokens(vocab, eot, sot, lb, n_lang, translate, transcribe, startoflm, startofprev, nospeech,
                           notimestamps, multi)
        if st.timestamp_begin + 1501 != vocab:
            raise AssertionError(f"timestamp layout mismatch for vocab {vocab}")
        return st


@dataclasses.dataclass
class GenerationSettings:
    """The generation_config fields the Whisper path reads (greedy decode, timestamps)."""

    special: SpecialTokens
    suppress_tokens: List[int]
    begin_suppress_tokens: List[int]
    max_initial_timestamp_index: Optional[int] = 50
    max_length: int = 448
    max_new_tokens: Optional[int] = None
    # generation_config.json's num_beams: what model.generate() uses when the call does not pass one (the ASR
    # pipeline callable overrides it with its own default 5, see pipeline.resolve_decode)
    num_beams: int = 1
    # False when a checkpoint's generation_config.json leaves max_length unset (GenerationConfig's global default
    # 20 then applies inside transformers, and the pipeline keeps its max_new_tokens=256)
    max_length_set: bool = True
    # token-level timestamps (return_timestamps="word"): cross-attention heads used for DTW and the median filter
    # width (generation_config.alignment_heads, config.median_filter_width)
    alignment_heads: Optional[List[Tuple[int, int]]] = None
    median_filter_width: int = 7
    # segment criteria of the temperature fallback when the call does not pass them (_set_thresholds_and_condition,
    # generation_whisper.py:1702-1730: the call's value, else generation_config's)
    compression_ratio_threshold: Optional[float] = None
    logprob_threshold: Optional[float] = None
    no_speech_threshold: Optional[float] = None
    # <|startofprev|> of condition_on_prev_tokens prompts (generation_config.prev_sot_token_id; None: transformers
    # falls back to suppress_tokens[-2], generation_whisper.py:1876-1881)
    prev_sot_token_id: Optional[int] = None

    @staticmethod
    def default(dims: WhisperDims) -> "GenerationSettings":
        st = SpecialTokens.for_vocab(dims.vocab)
        # Whisper checkpoints suppress a fixed list of punctuation / symbol tokens plus the
        # control tokens below (translate, transcribe, startoflm, startofprev, nospeech) and sot.
        # The synthetic default keeps that structure with a short symbol list.
        sym = [1, 2, 7, 8, 9, 10, 14, 25, 26, 27, 28, 29, 31, 58, 59, 60, 61, 62, 63, 90, 91, 92, 93]
        ctrl = [st.translate, st.transcribe, st.startoflm, st.startofprev, st.nospeech]
        # no published alignment heads for synthetic weights: every head of the upper half of the decoder (the
        # default of openai/whisper's model.py when a checkpoint ships none)
        heads = [(l, h) for l in range(dims.decoder_layers // 2, dims.decoder_layers) for h in range(dims.heads)]
        return GenerationSettings(special=st, suppress_tokens=sorted(set(sym + [st.sot] + ctrl)),
                                  begin_suppress_tokens=[220, st.eot], alignment_heads=heads)

    @staticmethod
    def from_checkpoint(path: str, dims: WhisperDims) -> "GenerationSettings":
        gs = GenerationSettings.default(dims)
        fn = os.path.join(path, "generation_config.json")
        if os.path.exists(fn):
            with open(fn) as f:
                cfg = json.load(f)
            if cfg.get("suppress_tokens") is not None:
                gs.suppress_tokens = list(cfg["suppress_tokens"])
            if cfg.get("begin_suppress_tokens") is not None:
                gs.begin_suppress_tokens = list(cfg["begin_suppress_tokens"])
            gs.max_initial_timestamp_index = cfg.get("max_initial_timestamp_index", gs.max_initial_timestamp_index)
            gs.max_length_set = cfg.get("max_length") is not None
            gs.max_length = cfg.get("max_length") or gs.max_length
            gs.num_beams = int(cfg.get("num_beams") or 1)
            if cfg.get("alignment_heads"):
                gs.alignment_heads = [(int(a), int(b)) for a, b in cfg["alignment_heads"]]
            if cfg.get("prev_sot_token_id") is not None:
                gs.prev_sot_token_id = int(cfg["prev_sot_token_id"])
            for k in ("compression_ratio_threshold", "logprob_threshold", "no_speech_threshold"):
                if cfg.get(k) is not None:
                    setattr(gs, k, float(cfg[k]))
        cfn = os.path.join(path, "config.json")
        if os.path.exists(cfn):
            with open(cfn) as f:
                gs.median_filter_width = int(json.load(f).get("median_filter_width", gs.median_filter_width))
        return gs

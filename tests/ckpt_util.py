"""Test helper: write a LOCAL Hugging Face Whisper checkpoint directory from the seeded synthetic weights (test
infrastructure; the product never imports this). The layout is what `transformers` itself reads and writes:
config.json + generation_config.json (written by WhisperConfig / GenerationConfig.save_pretrained),
model.safetensors (state-dict names of WhisperForConditionalGeneration, proj_out tied and not stored), and a
byte-level BPE tokenizer (vocab.json, merges.txt, added_tokens.json, special_tokens_map.json).

The vocabulary is the synthetic one with a block of ids replaced by byte-level encodings of multi-byte UTF-8 words, so
that decoding must join bytes across tokens; the checkpoint therefore decodes differently from the preset's vocabulary
and a test can tell which one was loaded."""
from __future__ import annotations

import json
import os
from typing import Dict, Optional

import numpy as np

from oracle import whisper_oracle as wo
from twamd.config import PRESETS, GenerationSettings
from twamd.tokenizer import bytes_to_unicode, special_token_strings, synthetic_vocab

# ids 300.. of the checkpoint vocabulary (replacing synthetic letter strings)
MULTIBYTE_WORDS = [" café", " naïve", " 日本", "語", " 😀", " niño", " —", " \"quoted\"", " Zürich", "ß", " ç",
                   " 한국어", " Ελληνικά", " ✓", "…", " Ωmega"]
MB_BASE = 300


def checkpoint_vocab(st) -> list:
    toks = synthetic_vocab(st)
    b2u = bytes_to_unicode()
    for k, w in enumerate(MULTIBYTE_WORDS):
        toks[MB_BASE + k] = "".join(b2u[b] for b in w.encode("utf-8"))
    assert len(set(toks[: st.eot])) == st.eot
    return toks


def write_tokenizer(path: str, st) -> None:
    toks = checkpoint_vocab(st)
    vocab = {t: i for i, t in enumerate(toks[: st.eot + 1])}  # real Whisper vocab.json ends with <|endoftext|>
    with open(os.path.join(path, "vocab.json"), "w", encoding="utf-8") as f:
        json.dump(vocab, f, ensure_ascii=False)
    # merges of the two-symbol tokens (each merge result is in the vocabulary; decoding never reads them)
    merges = ["#version: 0.2"] + [f"{t[0]} {t[1]}" for t in toks[256: st.eot] if len(t) == 2 and t[0] in vocab
                                  and t[1] in vocab][:64]
    with open(os.path.join(path, "merges.txt"), "w", encoding="utf-8") as f:
        f.write("\n".join(merges) + "\n")
    spec = special_token_strings(st)
    added = {spec[i]: i for i in range(st.eot + 1, st.vocab)}
    with open(os.path.join(path, "added_tokens.json"), "w", encoding="utf-8") as f:
        json.dump(added, f, ensure_ascii=False)
    with open(os.path.join(path, "special_tokens_map.json"), "w", encoding="utf-8") as f:
        json.dump({"bos_token": "<|endoftext|>", "eos_token": "<|endoftext|>", "unk_token": "<|endoftext|>",
                   "pad_token": "<|endoftext|>",
                   "additional_special_tokens": [spec[i] for i in range(st.eot + 1, st.timestamp_begin)]}, f)
    with open(os.path.join(path, "tokenizer_config.json"), "w", encoding="utf-8") as f:
        json.dump({"tokenizer_class": "WhisperTokenizer", "model_max_length": 1024, "add_prefix_space": False,
                   "errors": "replace"}, f)


def write_checkpoint(path: str, model: str = "test-mini", seed: int = 1234,
                     generation: Optional[Dict] = None, dtype=np.float32) -> str:
    """Write the checkpoint directory; `generation` overrides generation_config.json fields."""
    from safetensors.numpy import save_file
    from transformers import GenerationConfig, WhisperConfig

    d = PRESETS[model]
    gen = GenerationSettings.default(d)
    st = gen.special
    os.makedirs(path, exist_ok=True)
    WhisperConfig(vocab_size=d.vocab, num_mel_bins=d.n_mels, encoder_layers=d.encoder_layers,
                  encoder_attention_heads=d.heads, decoder_layers=d.decoder_layers, decoder_attention_heads=d.heads,
                  d_model=d.d_model, encoder_ffn_dim=d.ffn, decoder_ffn_dim=d.ffn, max_source_positions=1500,
                  max_target_positions=448, pad_token_id=st.eot, bos_token_id=st.eot, eos_token_id=st.eot,
                  decoder_start_token_id=st.sot, median_filter_width=7).save_pretrained(path)
    gc = dict(decoder_start_token_id=st.sot, eos_token_id=st.eot, pad_token_id=st.eot, bos_token_id=st.eot,
              no_timestamps_token_id=st.notimestamps, lang_to_id=st.lang_to_id(),
              task_to_id={"transcribe": st.transcribe, "translate": st.translate}, is_multilingual=st.is_multilingual,
              suppress_tokens=list(gen.suppress_tokens), begin_suppress_tokens=list(gen.begin_suppress_tokens),
              max_initial_timestamp_index=gen.max_initial_timestamp_index, max_length=448,
              alignment_heads=[list(h) for h in gen.alignment_heads])
    gc.update(generation or {})
    GenerationConfig(**gc).save_pretrained(path)
    sd = wo.synth_state_dict(d.d_model, d.encoder_layers, d.decoder_layers, d.ffn, d.n_mels, d.vocab, seed)
    save_file({k: np.ascontiguousarray(v.astype(dtype)) for k, v in sd.items()}, os.path.join(path, "model.safetensors"))
    write_tokenizer(path, st)
    return path


def decode_cases(st, n: int = 40, seed: int = 5):
    """Seeded id lists over the text vocabulary, biased towards the multi-byte block and the raw byte ids (so that
    UTF-8 sequences split across tokens, and invalid ones, occur)."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        k = int(rng.integers(1, 12))
        pool = rng.choice(3, size=k, p=[0.45, 0.35, 0.2])
        ids = []
        for p in pool:
            if p == 0:
                ids.append(MB_BASE + int(rng.integers(0, len(MULTIBYTE_WORDS))))
            elif p == 1:
                ids.append(int(rng.integers(0, 256)))
            else:
                ids.append(int(rng.integers(256, st.eot)))
        out.append(ids)
    # an é split over its two bytes, and a 4-byte emoji over four
    out.append([_byte_id(x) for x in "é".encode()])
    out.append([_byte_id(x) for x in "😀".encode()] + [MB_BASE])
    return out


def _byte_id(byte: int) -> int:
    """id of the single-byte token of `byte` in the synthetic vocabulary (ids < 256 are the byte symbols in table
    order)."""
    return list(bytes_to_unicode()).index(byte)

"""CPU BASELINE (test/bench infrastructure only): the reference's executed transcription path — the
transformers AutomaticSpeechRecognitionPipeline called with the reference's kwargs
(/root/reference/vocalis/core/audio_pipeline.py:351-358) — on the host CPU in fp32, with the same seeded
synthetic weights as the GPU engine and an in-memory tokenizer (no checkpoints exist offline).

Only bench.py's cpu_baseline leg (and tests) use this; it is never part of the product path.
"""
from __future__ import annotations

import os
import time
from typing import Dict, Optional

import numpy as np
import torch


def _hf_state_dict(dims, seed: int) -> Dict[str, torch.Tensor]:
    from oracle import whisper_oracle as wo

    sd = {k: torch.from_numpy(v) for k, v in wo.synth_state_dict(dims.d_model, dims.encoder_layers,
                                                                   dims.decoder_layers, dims.ffn, dims.n_mels,
                                                                   dims.vocab, seed).items()}
    sd["proj_out.weight"] = sd["model.decoder.embed_tokens.weight"]
    return sd


def build_pipeline(dims, gen, seed: int = 1234, threads: Optional[int] = None):
    from tokenizers import AddedToken
    from transformers import (AutomaticSpeechRecognitionPipeline, WhisperConfig, WhisperFeatureExtractor,
                              WhisperForConditionalGeneration, WhisperTokenizer)

    from twamd.tokenizer import special_token_strings, synthetic_vocab

    if threads:
        torch.set_num_threads(threads)
    st = gen.special
    cfg = WhisperConfig(vocab_size=dims.vocab, num_mel_bins=dims.n_mels, encoder_layers=dims.encoder_layers,
                        encoder_attention_heads=dims.heads, decoder_layers=dims.decoder_layers,
                        decoder_attention_heads=dims.heads, d_model=dims.d_model, encoder_ffn_dim=dims.ffn,
                        decoder_ffn_dim=dims.ffn, pad_token_id=st.eot, bos_token_id=st.eot, eos_token_id=st.eot,
                        decoder_start_token_id=st.sot, begin_suppress_tokens=None, suppress_tokens=None)
    with torch.device("meta"):
        m = WhisperForConditionalGeneration(cfg)
    m.load_state_dict(_hf_state_dict(dims, seed), strict=False, assign=True)
    m.proj_out.weight = m.model.decoder.embed_tokens.weight
    m.eval()
    gc = m.generation_config
    gc.decoder_start_token_id, gc.eos_token_id, gc.pad_token_id, gc.bos_token_id = st.sot, st.eot, st.eot, st.eot
    gc.no_timestamps_token_id = st.notimestamps
    gc.lang_to_id = st.lang_to_id()
    gc.task_to_id = {"transcribe": st.transcribe, "translate": st.translate}
    gc.is_multilingual = st.is_multilingual
    gc.suppress_tokens = list(gen.suppress_tokens)
    gc.begin_suppress_tokens = list(gen.begin_suppress_tokens)
    gc.max_initial_timestamp_index = gen.max_initial_timestamp_index
    gc.max_length = 448
    gc.forced_decoder_ids = None
    toks = synthetic_vocab(st)
    spec = special_token_strings(st)
    tk = WhisperTokenizer(vocab={t: i for i, t in enumerate(toks[: st.eot])}, merges=[],
                          additional_special_tokens=[spec[i] for i in range(st.eot + 1, st.timestamp_begin)],
                          pad_token="<|endoftext|>")
    tk.add_tokens([AddedToken(spec[i], special=False, normalized=False) for i in range(st.timestamp_begin, st.vocab)])
    fe = WhisperFeatureExtractor(feature_size=dims.n_mels)
    return AutomaticSpeechRecognitionPipeline(model=m, feature_extractor=fe, tokenizer=tk, device=-1)


def time_reference(dims, gen, audio: np.ndarray, max_new_tokens: int, threads: int, seed: int = 1234,
                   num_beams: int = 1, one_pass: bool = False, chunk_length_s: float = 60,
                   stride_length_s: float = 5, pipe=None) -> dict:
    """Wall time of the ASR pipeline call on `audio` (default: the reference kwargs chunk 60 / stride 5 /
    batch 32, vocalis/core/audio_pipeline.py:351-358). one_pass: generation_config.force_unique_generate_call
    (a single seek pass per window). pipe: a pipeline from build_pipeline to reuse (weights are built once)."""
    if pipe is None:
        pipe = build_pipeline(dims, gen, seed, threads)
    if one_pass:
        pipe.generation_config.force_unique_generate_call = True
    t0 = time.perf_counter()
    with torch.no_grad():
        out = pipe(audio.copy(), chunk_length_s=chunk_length_s, batch_size=32, stride_length_s=stride_length_s,
                   generate_kwargs={"task": "transcribe", "num_beams": num_beams, "max_new_tokens": max_new_tokens},
                   return_timestamps=True)
    wall = time.perf_counter() - t0
    return {"wall_s": wall, "audio_s": len(audio) / 16000.0, "threads": threads, "n_chars": len(out["text"])}

"""Generate the golden vectors that pin oracle/ and the host logic to the reference's executed code.

Runs transformers (5.15.0 here; the reference's hot path is transformers' Whisper, not vendored in
/root/reference) on CPU in float32 with the seeded synthetic weights of oracle/whisper_oracle.py and an
in-memory tokenizer built from twamd.tokenizer.synthetic_vocab, then stores small fixtures:

  logmel.npz        WhisperFeatureExtractor features (128 and 80 mels) of synthetic clips, subsampled
  model.npz         test-mini encoder output rows, teacher-forced decoder logits top-k, generate() tokens
  pipeline.json     AutomaticSpeechRecognitionPipeline outputs with the reference's call kwargs
                    (vocalis/core/audio_pipeline.py:351-358, num_beams=1 for greedy parity) and 30-s mode
  decode_asr.json   tokenizer._decode_asr on seeded random strided token sequences
  word.npz/.json    token-level timestamps (cross-attention DTW) of generate(return_token_timestamps=True) and
                    the pipeline's return_timestamps="word" output, plus HF's _median_filter / _dynamic_time_warping
                    on seeded random matrices
  beam_word.json    token-level timestamps with beam search (generate() token times, pipeline word chunks)
  fallback_beam.json  the temperature-fallback criteria and outcomes with beam search (num_beams=3)
  word_combos.json  word timestamps with long-form input / condition_on_prev_tokens / the fallback criteria, and
                    the fallback with beam search (pipeline outputs)
  longform.json     long-form (unchunked > 30 s) pipeline outputs and condition_on_prev_tokens, with every seek
                    pass's decoder prompt and raw output (spied from generate_with_fallback)
  fallback.json     the temperature-fallback criteria (compression ratio, avg logprob, no-speech probability) of
                    every seek pass and a deterministic no-speech skip, spied from transformers' generate()
  tiny.npz          whisper-tiny.en (configs[0], English-only) encoder rows, teacher-forced logits, generate() passes
                    with their processed top-16 scores
  beam.json         generate(num_beams=5) token sequences (the pipeline's default decode, asr:160-163) of
                    test-mini on three windows, with and without timestamps and with a max_length stop
  beam_long.json    the reference's call (default beam-5) on 8 minutes of audio at test-mini (50 beam rows per batch)
  options.json      the ASR pipeline with translate (reference call), no timestamps, a forced language, return_language
  sweep.json        the ASR pipeline over chunk / stride / batch / beam / timestamp / task / language variations
  edge.json         the ASR pipeline on empty and sub-frame inputs (outputs or the exception transcribe() wraps)
  large_v3.npz      whisper-large-v3 dims (the reference's default model: 32-layer decoder): encoder rows,
                    teacher-forced logits, generate() passes with processed top-16 scores
  turbo_word.npz    generate(return_token_timestamps=True) at large-v3-turbo dims with the default alignment heads
  turbo_beam.npz    generate(num_beams=5) at large-v3-turbo dims, with and without timestamps: the 5 finished
                    hypotheses and their beam scores (oracle beam search on the fp32 model's logits, checked to
                    return generate()'s best hypothesis)

Usage: python tests/golden/make_golden.py   (≈1-2 min on 8 CPU cores)
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "turbo-whisper-workspace_amd"))

from oracle import whisper_oracle as wo  # noqa: E402
from twamd.config import PRESETS, GenerationSettings  # noqa: E402
from twamd.synth_audio import silence, speech_like, white_noise  # noqa: E402
from twamd.tokenizer import special_token_strings, synthetic_vocab  # noqa: E402

SEED = 1234
DIMS = PRESETS["test-mini"]


def hf_tokenizer(st):
    from tokenizers import AddedToken
    from transformers import WhisperTokenizer

    toks = synthetic_vocab(st)
    vocab = {t: i for i, t in enumerate(toks[: st.eot])}
    spec = special_token_strings(st)
    add = [spec[i] for i in range(st.eot + 1, st.timestamp_begin)]
    tk = WhisperTokenizer(vocab=vocab, merges=[], additional_special_tokens=add, pad_token="<|endoftext|>")
    tk.add_tokens([AddedToken(spec[i], special=False, normalized=False) for i in range(st.timestamp_begin, st.vocab)])
    assert tk.convert_tokens_to_ids("<|notimestamps|>") == st.notimestamps
    assert sorted(tk.all_special_ids) == st.special_ids()
    return tk


def hf_model(dims, sd_np, gen):
    from transformers import WhisperConfig, WhisperForConditionalGeneration

    st = gen.special
    cfg = WhisperConfig(vocab_size=dims.vocab, num_mel_bins=dims.n_mels, encoder_layers=dims.encoder_layers,
                        encoder_attention_heads=dims.heads, decoder_layers=dims.decoder_layers,
                        decoder_attention_heads=dims.heads, d_model=dims.d_model, encoder_ffn_dim=dims.ffn,
                        decoder_ffn_dim=dims.ffn, max_source_positions=1500, max_target_positions=448,
                        pad_token_id=st.eot, bos_token_id=st.eot, eos_token_id=st.eot,
                        decoder_start_token_id=st.sot, begin_suppress_tokens=None, suppress_tokens=None)
    cfg._attn_implementation = "eager"
    m = WhisperForConditionalGeneration(cfg).eval()
    sd = {k: torch.from_numpy(v.copy()) for k, v in sd_np.items()}
    sd["proj_out.weight"] = sd["model.decoder.embed_tokens.weight"]
    missing, unexpected = m.load_state_dict(sd, strict=False)
    assert not unexpected, unexpected
    assert all(k == "proj_out.weight" for k in missing), missing
    gc = m.generation_config
    gc.decoder_start_token_id = st.sot
    gc.eos_token_id = st.eot
    gc.pad_token_id = st.eot
    gc.bos_token_id = st.eot
    gc.no_timestamps_token_id = st.notimestamps
    gc.lang_to_id = st.lang_to_id()
    gc.task_to_id = {"transcribe": st.transcribe, "translate": st.translate}
    gc.is_multilingual = st.is_multilingual
    gc.suppress_tokens = list(gen.suppress_tokens)
    gc.begin_suppress_tokens = list(gen.begin_suppress_tokens)
    gc.max_initial_timestamp_index = gen.max_initial_timestamp_index
    gc.max_length = 448
    gc.forced_decoder_ids = None
    return m


def clips():
    return {"speech30": speech_like(30.0, 1234), "noise12": white_noise(12.3, 7), "zeros30": silence(30.0),
            "speech45": speech_like(45.0, 99)}


def make_logmel(out):
    from transformers import WhisperFeatureExtractor

    res = {}
    for n_mels in (128, 80):
        fe = WhisperFeatureExtractor(feature_size=n_mels)
        for name, x in clips().items():
            if n_mels == 80 and name != "speech30":
                continue
            f = fe(x, sampling_rate=16000, return_tensors="np")["input_features"][0]
            res[f"feat{n_mels}_{name}_sub"] = f[:, ::15].astype(np.float32)
            res[f"feat{n_mels}_{name}_rowsum"] = f.sum(axis=1).astype(np.float64)
    np.savez_compressed(os.path.join(out, "logmel.npz"), **res)


def make_model(out):
    from transformers import WhisperFeatureExtractor

    d = DIMS
    gen = GenerationSettings.default(d)
    st = gen.special
    sd = wo.synth_state_dict(d.d_model, d.encoder_layers, d.decoder_layers, d.ffn, d.n_mels, d.vocab, SEED)
    m = hf_model(d, sd, gen)
    fe = WhisperFeatureExtractor(feature_size=d.n_mels)
    cl = clips()
    feats = np.stack([fe(cl[k], sampling_rate=16000, return_tensors="np")["input_features"][0]
                      for k in ("speech30", "noise12")])
    res = {}
    with torch.no_grad():
        enc = m.model.encoder(torch.from_numpy(feats)).last_hidden_state.numpy()
    res["enc_rows_idx"] = np.array([0, 1, 750, 1499])
    res["enc_rows"] = enc[:, [0, 1, 750, 1499]].astype(np.float32)
    res["enc_mean"] = enc.mean(axis=(1, 2))
    res["enc_std"] = enc.std(axis=(1, 2))
    # generate (short-form, timestamps, greedy) for both clips
    with torch.no_grad():
        gen_out = m.generate(torch.from_numpy(feats), task="transcribe", return_timestamps=True, num_beams=1,
                             max_new_tokens=40, return_segments=True)
    seqs = gen_out["sequences"].numpy()
    res["gen_sequences"] = seqs
    # detected language + teacher-forced logits along the first segment pass of clip 0
    with torch.no_grad():
        lang = m.detect_language(input_features=torch.from_numpy(feats)).numpy()
    res["gen_lang"] = lang
    first = gen_out["segments"][0][0]["result"]
    full = first["sequences"] if isinstance(first, dict) else first
    full = full.numpy().reshape(-1)
    res["tf_input_ids"] = full[:24]
    with torch.no_grad():
        lg = m(input_features=torch.from_numpy(feats[:1]), decoder_input_ids=torch.from_numpy(full[None, :24])).logits[0]
    lg = lg.numpy()
    top = np.argsort(-lg, axis=1, kind="stable")[:, :16]
    res["tf_top_idx"] = top
    res["tf_top_val"] = np.take_along_axis(lg, top, 1).astype(np.float32)
    res["tf_lse"] = (np.log(np.exp(lg - lg.max(1, keepdims=True)).sum(1)) + lg.max(1)).astype(np.float64)
    res["tf_ts_slice"] = lg[:, st.timestamp_begin: st.timestamp_begin + 64].astype(np.float32)
    np.savez_compressed(os.path.join(out, "model.npz"), **res)


def make_pipeline(out):
    from transformers import AutomaticSpeechRecognitionPipeline, WhisperFeatureExtractor

    d = DIMS
    gen = GenerationSettings.default(d)
    sd = wo.synth_state_dict(d.d_model, d.encoder_layers, d.decoder_layers, d.ffn, d.n_mels, d.vocab, SEED)
    m = hf_model(d, sd, gen)
    tk = hf_tokenizer(gen.special)
    fe = WhisperFeatureExtractor(feature_size=d.n_mels)
    pipe = AutomaticSpeechRecognitionPipeline(model=m, feature_extractor=fe, tokenizer=tk, device=-1)
    audio = np.concatenate([speech_like(40.0, 5), white_noise(35.0, 11)])  # 75 s
    cases = []
    for name, kw in [
        ("ref_60_5", dict(chunk_length_s=60, stride_length_s=5, batch_size=32)),
        ("mode_30_0", dict(chunk_length_s=30, stride_length_s=0, batch_size=2)),
        ("short_nochunk", dict()),
    ]:
        x = audio if name != "short_nochunk" else audio[: 20 * 16000]
        r = pipe(x.copy(), generate_kwargs={"task": "transcribe", "num_beams": 1, "max_new_tokens": 40},
                 return_timestamps=True, **kw)
        cases.append({"name": name, "kwargs": kw, "n_samples": int(len(x)), "output": _jsonable(r)})
    with open(os.path.join(out, "pipeline.json"), "w") as f:
        json.dump({"seed": SEED, "dims": "test-mini", "audio": "speech_like(40,5)+white_noise(35,11)",
                   "cases": cases}, f, indent=1)


def make_decode_asr(out):
    from transformers.models.whisper.tokenization_whisper import _decode_asr

    gen = GenerationSettings.default(PRESETS["large-v3-turbo"])
    st = gen.special
    tk = hf_tokenizer(st)
    rng = np.random.Generator(np.random.PCG64(2024))
    cases = []
    for ci in range(40):
        n_chunks = int(rng.integers(1, 5))
        chunk_len, left, right = (60.0, 5.0, 5.0) if ci % 2 == 0 else (30.0, 0.0, 0.0)
        outputs = []
        for k in range(n_chunks):
            toks = []
            t = int(rng.integers(0, 50))
            if ci % 5 == 3:
                toks.append(st.lang_begin + int(rng.integers(0, 5)))
            for _ in range(int(rng.integers(0, 6))):
                toks.append(st.timestamp_begin + t)
                toks += [int(v) for v in rng.integers(256, 3000, size=int(rng.integers(0, 6)))]
                t = min(1500, t + int(rng.integers(0, 400)))
                toks.append(st.timestamp_begin + t)
                if rng.random() < 0.3:
                    t = min(1500, t + int(rng.integers(0, 50)))
            if rng.random() < 0.3:
                toks += [int(v) for v in rng.integers(256, 3000, size=3)]
            if rng.random() < 0.4:
                toks += [st.eot] * int(rng.integers(1, 3))
            is_first, is_last = k == 0, k == n_chunks - 1
            stride = (chunk_len if not is_last else chunk_len * float(rng.uniform(0.3, 1.0)),
                      0.0 if is_first else left, 0.0 if is_last else right)
            outputs.append({"tokens": toks, "stride": stride})
        rt = bool(ci % 7 != 6)
        hf_outs = [{"tokens": torch.tensor([o["tokens"]], dtype=torch.long), "stride": o["stride"]} for o in outputs]
        text, opt = _decode_asr(tk, hf_outs, return_timestamps=rt, return_language=(ci % 5 == 3),
                                time_precision=0.02)
        cases.append({"outputs": outputs, "return_timestamps": rt, "return_language": ci % 5 == 3,
                      "text": text, "optional": _jsonable(opt)})
    with open(os.path.join(out, "decode_asr.json"), "w") as f:
        json.dump(cases, f)


def make_beam(out):
    from transformers import WhisperFeatureExtractor

    d = DIMS
    gen = GenerationSettings.default(d)
    sd = wo.synth_state_dict(d.d_model, d.encoder_layers, d.decoder_layers, d.ffn, d.n_mels, d.vocab, SEED)
    m = hf_model(d, sd, gen)
    fe = WhisperFeatureExtractor(feature_size=d.n_mels)
    cl = clips()
    names = ["speech30", "noise12", "zeros30"]
    feats = np.stack([fe(cl[k], sampling_rate=16000, return_tensors="np")["input_features"][0] for k in names])
    cases = []
    for ts, mnt in ((True, 40), (False, 40), (True, 9)):
        with torch.no_grad():
            o = m.generate(torch.from_numpy(feats), task="transcribe", return_timestamps=ts, num_beams=5,
                           max_new_tokens=mnt)
        seqs = o["sequences"] if isinstance(o, dict) else o
        cases.append({"return_timestamps": ts, "max_new_tokens": mnt, "clips": names,
                      "sequences": seqs.numpy().tolist()})
    # the ASR pipeline with the reference's call and its default decode (num_beams=5)
    from transformers import AutomaticSpeechRecognitionPipeline

    tk = hf_tokenizer(gen.special)
    pipe = AutomaticSpeechRecognitionPipeline(model=m, feature_extractor=fe, tokenizer=tk, device=-1)
    audio = np.concatenate([speech_like(40.0, 5), white_noise(35.0, 11)])  # 75 s
    pcases = []
    for name, kw in [("ref_60_5", dict(chunk_length_s=60, stride_length_s=5, batch_size=32)),
                     ("mode_30_0", dict(chunk_length_s=30, stride_length_s=0, batch_size=2))]:
        r = pipe(audio.copy(), generate_kwargs={"task": "transcribe", "num_beams": 5, "max_new_tokens": 40},
                 return_timestamps=True, **kw)
        pcases.append({"name": name, "kwargs": kw, "output": _jsonable(r)})
    with open(os.path.join(out, "beam.json"), "w") as f:
        json.dump({"seed": SEED, "dims": "test-mini", "num_beams": 5, "cases": cases,
                   "pipeline_audio": "speech_like(40,5)+white_noise(35,11)", "pipeline": pcases}, f)


ALIGN_HEADS_MINI = [[1, 0], [1, 1], [1, 2], [1, 3]]  # test-mini: every head of the upper half of the decoder


def make_word(out):
    from transformers import AutomaticSpeechRecognitionPipeline, WhisperFeatureExtractor
    from transformers.models.whisper.generation_whisper import _dynamic_time_warping, _median_filter

    res = {}
    rng = np.random.default_rng(77)
    for k, (n, m) in enumerate(((5, 40), (17, 300), (1, 9), (30, 30))):
        mat = rng.standard_normal((n, m))
        ti, tj = _dynamic_time_warping(mat)
        res[f"dtw{k}_in"], res[f"dtw{k}_text"], res[f"dtw{k}_time"] = mat, ti, tj
    x = rng.standard_normal((2, 3, 11, 50)).astype(np.float32)
    res["median_in"], res["median_out"] = x, _median_filter(torch.from_numpy(x), 7).numpy()
    d = DIMS
    gen = GenerationSettings.default(d)
    sd = wo.synth_state_dict(d.d_model, d.encoder_layers, d.decoder_layers, d.ffn, d.n_mels, d.vocab, SEED)
    m = hf_model(d, sd, gen)
    m.generation_config.alignment_heads = ALIGN_HEADS_MINI
    fe = WhisperFeatureExtractor(feature_size=d.n_mels)
    cl = clips()
    for name in ("speech30", "noise12"):
        f = fe(cl[name], sampling_rate=16000, return_tensors="pt", return_attention_mask=True)
        with torch.no_grad():
            o = m.generate(f["input_features"], attention_mask=f["attention_mask"], task="transcribe",
                           return_timestamps=True, return_token_timestamps=True, max_new_tokens=40)
        res[f"gen_{name}_seq"] = o["sequences"].numpy()
        res[f"gen_{name}_ts"] = o["token_timestamps"].numpy()
    np.savez_compressed(os.path.join(out, "word.npz"), **res)
    tk = hf_tokenizer(gen.special)
    pipe = AutomaticSpeechRecognitionPipeline(model=m, feature_extractor=fe, tokenizer=tk, device=-1)
    audio = np.concatenate([speech_like(40.0, 5), white_noise(35.0, 11)])  # 75 s
    cases = []
    for name, x, kw in (("single_20s", audio[: 20 * 16000], {}),
                        ("mode_30_0", audio, dict(chunk_length_s=30, stride_length_s=0, batch_size=8))):
        r = pipe(x.copy(), generate_kwargs={"task": "transcribe", "num_beams": 1, "max_new_tokens": 40},
                 return_timestamps="word", **kw)
        cases.append({"name": name, "kwargs": kw, "n_samples": int(len(x)), "output": _jsonable(r)})
    with open(os.path.join(out, "word.json"), "w") as f:
        json.dump({"seed": SEED, "dims": "test-mini", "alignment_heads": ALIGN_HEADS_MINI,
                   "audio": "speech_like(40,5)+white_noise(35,11)", "cases": cases}, f)


def make_beam_word(out):
    """Token-level timestamps with beam search (return_timestamps="word" / return_token_timestamps with num_beams=3,
    the alignment-head cross-attentions gathered along each hypothesis' beam_indices, generation_whisper.py:265-300):
    generate() sequences + token times of two clips, and the ASR pipeline's word chunks (single window, 30-s mode)."""
    from transformers import AutomaticSpeechRecognitionPipeline, WhisperFeatureExtractor

    d = DIMS
    gen = GenerationSettings.default(d)
    sd = wo.synth_state_dict(d.d_model, d.encoder_layers, d.decoder_layers, d.ffn, d.n_mels, d.vocab, SEED)
    m = hf_model(d, sd, gen)
    m.generation_config.alignment_heads = ALIGN_HEADS_MINI
    fe = WhisperFeatureExtractor(feature_size=d.n_mels)
    cl = clips()
    gens = []
    for name in ("speech30", "noise12"):
        f = fe(cl[name], sampling_rate=16000, return_tensors="pt", return_attention_mask=True)
        with torch.no_grad():
            o = m.generate(f["input_features"], attention_mask=f["attention_mask"], task="transcribe", num_beams=3,
                           return_timestamps=True, return_token_timestamps=True, max_new_tokens=24)
        gens.append({"clip": name, "sequences": o["sequences"].tolist(), "token_timestamps": o["token_timestamps"].tolist()})
    pipe = AutomaticSpeechRecognitionPipeline(model=m, feature_extractor=fe, tokenizer=hf_tokenizer(gen.special),
                                              device=-1)
    audio = np.concatenate([speech_like(40.0, 5), white_noise(35.0, 11)])
    cases = []
    for name, x, kw in (("single_20s_beam3", audio[: 20 * 16000], {}),
                        ("mode_30_0_beam3", audio, dict(chunk_length_s=30, stride_length_s=0, batch_size=3))):
        r = pipe(x.copy(), generate_kwargs={"task": "transcribe", "num_beams": 3, "max_new_tokens": 24},
                 return_timestamps="word", **kw)
        cases.append({"name": name, "kwargs": kw, "n_samples": int(len(x)), "output": _jsonable(r)})
    with open(os.path.join(out, "beam_word.json"), "w") as f:
        json.dump({"seed": SEED, "dims": "test-mini", "alignment_heads": ALIGN_HEADS_MINI, "num_beams": 3,
                   "generate": gens, "cases": cases}, f)


WORD_COMBO_CASES = [  # name, pipeline kwargs, generate_kwargs, return_timestamps
    ("long_word", {}, {"task": "transcribe", "num_beams": 1, "max_new_tokens": 40}, "word"),
    ("cond_word", dict(chunk_length_s=30, stride_length_s=0, batch_size=3),
     {"task": "transcribe", "num_beams": 1, "max_new_tokens": 40, "condition_on_prev_tokens": True}, "word"),
    ("fallback_word", dict(chunk_length_s=30, stride_length_s=0, batch_size=3),
     {"task": "transcribe", "num_beams": 1, "max_new_tokens": 40, "temperature": (0.0,), "logprob_threshold": -3.0,
      "no_speech_threshold": 3e-5}, "word"),
    ("fallback_beam3", dict(chunk_length_s=30, stride_length_s=0, batch_size=3),
     {"task": "transcribe", "num_beams": 3, "max_new_tokens": 24, "temperature": (0.0,), "logprob_threshold": -3.0,
      "no_speech_threshold": 3e-5}, True),
    ("long_cond_word", {}, {"task": "transcribe", "num_beams": 1, "max_new_tokens": 40,
                            "condition_on_prev_tokens": True}, "word"),
]


def make_word_combos(out):
    """The ASR pipeline at test-mini (alignment heads ALIGN_HEADS_MINI) on 75 s of audio with the call options
    combined: word timestamps on a long-form input, with condition_on_prev_tokens, with the fallback criteria (one
    temperature: deterministic), and the fallback with beam search."""
    from transformers import AutomaticSpeechRecognitionPipeline, WhisperFeatureExtractor

    d = DIMS
    gen = GenerationSettings.default(d)
    sd = wo.synth_state_dict(d.d_model, d.encoder_layers, d.decoder_layers, d.ffn, d.n_mels, d.vocab, SEED)
    m = hf_model(d, sd, gen)
    m.generation_config.alignment_heads = ALIGN_HEADS_MINI
    fe = WhisperFeatureExtractor(feature_size=d.n_mels)
    pipe = AutomaticSpeechRecognitionPipeline(model=m, feature_extractor=fe, tokenizer=hf_tokenizer(gen.special),
                                              device=-1)
    audio = np.concatenate([speech_like(40.0, 5), white_noise(35.0, 11)]).astype(np.float32)
    res = []
    for name, kw, gk, ts in WORD_COMBO_CASES:
        c = {"name": name, "kwargs": kw, "generate_kwargs": gk, "return_timestamps": ts}
        try:
            c["output"] = _jsonable(pipe(audio.copy(), generate_kwargs=dict(gk), return_timestamps=ts, **kw))
        except Exception as e:  # noqa: BLE001 - recorded as the reference would surface it
            c["error"] = {"type": type(e).__name__, "message": str(e)}
        res.append(c)
    with open(os.path.join(out, "word_combos.json"), "w") as f:
        json.dump({"dims": "test-mini", "alignment_heads": ALIGN_HEADS_MINI,
                   "audio": "speech_like(40,5)+white_noise(35,11)", "cases": res}, f)


def make_defaults(out):
    """The decode the ASR pipeline actually runs (num_beams / max_new_tokens reaching model.generate) for
    checkpoint generation configs x call kwargs: Pipeline.__init__'s default-config resolution ($TF/pipelines/
    base.py:887-908) and _forward's generate call (automatic_speech_recognition.py:483-529)."""
    from transformers import AutomaticSpeechRecognitionPipeline, WhisperFeatureExtractor

    d = DIMS
    gen = GenerationSettings.default(d)
    sd = wo.synth_state_dict(d.d_model, d.encoder_layers, d.decoder_layers, d.ffn, d.n_mels, d.vocab, SEED)
    fe = WhisperFeatureExtractor(feature_size=d.n_mels)
    tk = hf_tokenizer(gen.special)
    ckpts = {"whisper_default": {}, "num_beams_1": {"num_beams": 1}, "num_beams_3": {"num_beams": 3},
             "no_max_length": {"max_length": None}, "max_new_tokens_64": {"max_new_tokens": 64}}
    calls = {"reference_call": {"task": "transcribe"}, "greedy": {"task": "transcribe", "num_beams": 1},
             "mnt_40": {"task": "transcribe", "max_new_tokens": 40}}
    cases = []
    for cname, cfg in ckpts.items():
        m = hf_model(d, sd, gen)
        for k, v in cfg.items():
            setattr(m.generation_config, k, v)
        pipe = AutomaticSpeechRecognitionPipeline(model=m, feature_extractor=fe, tokenizer=tk, device=-1)
        seen = {}

        def spy(*a, _orig=m.generate, **kw):
            gc = kw["generation_config"]
            seen.update(num_beams=kw.get("num_beams", gc.num_beams),
                        max_new_tokens=kw.get("max_new_tokens", gc.max_new_tokens),
                        max_length=kw.get("max_length", gc.max_length))
            raise StopIteration  # the resolved values are all that is wanted

        m.generate = spy
        for kname, kw in calls.items():
            seen.clear()
            try:
                pipe(np.zeros(16000, np.float32), generate_kwargs=dict(kw), return_timestamps=True)
            except (StopIteration, RuntimeError):
                pass
            cases.append({"checkpoint_generation_config": cfg, "generate_kwargs": kw, "resolved": dict(seen)})
    with open(os.path.join(out, "defaults.json"), "w") as f:
        json.dump({"transformers": __import__("transformers").__version__, "cases": cases}, f, indent=1)


def make_ckpt(out):
    """transformers' WhisperTokenizer loaded FROM a checkpoint directory written by tests/ckpt_util.py (byte-level
    vocab.json with multi-byte UTF-8 tokens, merges.txt, added_tokens.json): decode() of seeded id lists, and the
    special-token layout it reports."""
    import tempfile

    from transformers import WhisperTokenizer

    sys.path.insert(0, os.path.dirname(HERE))
    import ckpt_util as cu

    st = GenerationSettings.default(DIMS).special
    with tempfile.TemporaryDirectory() as d:
        cu.write_tokenizer(d, st)
        tk = WhisperTokenizer.from_pretrained(d)
        cases = [{"ids": ids, "text": tk.decode(ids)} for ids in cu.decode_cases(st)]
        layout = {k: tk.convert_tokens_to_ids(k) for k in ("<|endoftext|>", "<|startoftranscript|>", "<|en|>",
                                                           "<|transcribe|>", "<|notimestamps|>", "<|0.00|>",
                                                           "<|30.00|>")}
        special = sorted(tk.all_special_ids)
    with open(os.path.join(out, "ckpt_decode.json"), "w", encoding="utf-8") as f:
        json.dump({"transformers": __import__("transformers").__version__, "vocab_size": len(tk), "layout": layout,
                   "all_special_ids": special, "cases": cases}, f, ensure_ascii=False)


TURBO_CLIPS = ("speech30", "noise12")
TURBO_BENCH_WINDOWS = (0, 23)   # bench.py's rank-0 workload(24): window 0 speech_like(30, 1234), window 23 silent


def _passes_from_segments(segs, prompt_len):
    """Raw generated tokens (prompt stripped, trailing pads/EOS kept as generated) of every seek pass, from
    generate(return_segments=True): consecutive segments of one pass share its `result` sequence."""
    passes, last = [], None
    for s in segs:
        r = s["result"]
        if last is not None and r is last:
            continue
        last = r
        r = (r["sequences"] if isinstance(r, dict) else r).reshape(-1)
        passes.append([int(t) for t in r[prompt_len:].tolist()])
    return passes


def _teacher_forced_pass_scores(m, feats, seek, prompt, toks, g, use_ts=True, k=16):
    """transformers' logits along one seek pass (features sliced at `seek` and zero-padded, as _get_input_segment
    does), run through the processor chain (oracle.process_logits, itself pinned to transformers' processors by
    the test-mini goldens): per step the top-k processed scores and the timestamp-rule margin. These let a
    device decode be checked within a stated tolerance at its first divergence from the fp32 sequence."""
    seg = np.zeros_like(feats)
    seg[:, : 3000 - seek] = feats[:, seek:]
    ids = list(prompt) + [t for t in toks]
    with torch.no_grad():
        lg = m(input_features=torch.from_numpy(seg[None]), decoder_input_ids=torch.tensor([ids[:-1] if toks else ids])
               ).logits[0].numpy()
    lg = lg[len(prompt) - 1:]
    top_i, top_v, margin = [], [], []
    for t in range(len(toks)):
        s = wo.process_logits(lg[t], toks[:t], g, use_ts)
        order = np.argsort(-s, kind="stable")[:k]
        top_i.append(order)
        top_v.append(s[order])
        margin.append(wo._ts_rule_margin(wo.process_logits_no_rule(lg[t], toks[:t], g), g.ts_begin) if use_ts else 0.0)
    return (np.array(top_i, np.int32).reshape(-1, k), np.array(top_v, np.float32).reshape(-1, k),
            np.array(margin, np.float32))


def make_turbo(out):
    """large-v3-turbo dims (d 1280, 32 + 4 layers, 20 heads, vocab 51866) with the seeded synthetic weights: the
    encoder output, teacher-forced logits, generate() tokens + language, and bench.py's first-pass decode of two
    of its windows (EOS suppressed, 128 new tokens), all from transformers on CPU fp32."""
    from transformers import WhisperFeatureExtractor
    from twamd.synth_audio import workload

    d = PRESETS["large-v3-turbo"]
    gen = GenerationSettings.default(d)
    st = gen.special
    g = wo.GenCfg(d.vocab, st.eot, st.sot, st.lang_begin, st.n_languages, st.transcribe, st.translate,
                  st.notimestamps, gen.suppress_tokens, gen.begin_suppress_tokens)
    sd = wo.synth_state_dict(d.d_model, d.encoder_layers, d.decoder_layers, d.ffn, d.n_mels, d.vocab, SEED)
    m = hf_model(d, sd, gen)
    del sd
    fe = WhisperFeatureExtractor(feature_size=d.n_mels)
    cl = clips()
    feats = np.stack([fe(cl[k], sampling_rate=16000, return_tensors="np")["input_features"][0] for k in TURBO_CLIPS])
    res = {}
    with torch.no_grad():
        enc = m.model.encoder(torch.from_numpy(feats)).last_hidden_state.numpy()
    res["enc_rows_idx"] = np.array([0, 1, 2, 375, 750, 1124, 1498, 1499])
    res["enc_rows"] = enc[:, res["enc_rows_idx"]].astype(np.float32)
    res["enc_mean"] = enc.mean(axis=(1, 2))
    res["enc_std"] = enc.std(axis=(1, 2))
    res["enc_row_norm"] = np.linalg.norm(enc, axis=2).astype(np.float32)      # [2][1500]
    res["enc_col_mean"] = enc.mean(axis=1).astype(np.float32)                 # [2][1280]
    del enc
    with torch.no_grad():
        lang = m.detect_language(input_features=torch.from_numpy(feats)).numpy()
    res["gen_lang"] = lang
    with torch.no_grad():
        o = m.generate(torch.from_numpy(feats), task="transcribe", return_timestamps=True, num_beams=1,
                       max_new_tokens=40, return_segments=True)
    res["gen_sequences"] = o["sequences"].numpy()
    for i in range(len(TURBO_CLIPS)):
        passes = _passes_from_segments(o["segments"][i], 3)
        pr = [st.sot, int(lang[i]), st.transcribe]
        seek, ti, tv, mg, kept = 0, [], [], [], []
        offs = [0]
        for p in passes:
            toks = p[: p.index(st.eot) + 1] if st.eot in p else p
            a, b, c = _teacher_forced_pass_scores(m, feats[i], seek, pr, toks, g)
            ti.append(a); tv.append(b); mg.append(c)
            seq = toks[:-1] if toks and toks[-1] == st.eot else toks
            seg, off = wo.retrieve_segment(seq, 3000 - seek, g.ts_begin)
            kept += seg
            seek += off
            offs.append(seek)
        ref = [int(t) for t in res["gen_sequences"][i]]
        while ref and ref[-1] == st.eot:
            ref.pop()
        assert kept == ref, ("pass reconstruction differs from generate()", i)
        res[f"gen{i}_pass_len"] = np.array([len(x) for x in ti], np.int32)
        res[f"gen{i}_pass_tokens"] = np.concatenate(
            [np.array(p[: len(x)], np.int32) for p, x in zip(passes, ti)]) if passes else np.zeros(0, np.int32)
        res[f"gen{i}_pass_seek"] = np.array(offs[:-1], np.int32)
        res[f"gen{i}_top_idx"], res[f"gen{i}_top_val"] = np.concatenate(ti), np.concatenate(tv)
        res[f"gen{i}_ts_margin"] = np.concatenate(mg)
    # teacher-forced raw logits along clip 0's first pass (24 positions), as test-mini's model.npz
    p0 = [st.sot, int(lang[0]), st.transcribe] + [int(t) for t in res["gen0_pass_tokens"][:21]]
    res["tf_input_ids"] = np.array(p0[:24])
    with torch.no_grad():
        lg = m(input_features=torch.from_numpy(feats[:1]), decoder_input_ids=torch.tensor([p0[:24]])).logits[0].numpy()
    top = np.argsort(-lg, axis=1, kind="stable")[:, :16]
    res["tf_top_idx"] = top
    res["tf_top_val"] = np.take_along_axis(lg, top, 1).astype(np.float32)
    res["tf_lse"] = (np.log(np.exp(lg - lg.max(1, keepdims=True)).sum(1)) + lg.max(1)).astype(np.float64)
    # bench.py's decode: EOS suppressed, 128 new tokens, first seek pass only (max_passes=1)
    wl = workload(24, 30.0, seed=1234)
    bfeats = np.stack([fe(wl[w], sampling_rate=16000, return_tensors="np")["input_features"][0]
                       for w in TURBO_BENCH_WINDOWS])
    gb = wo.GenCfg(d.vocab, st.eot, st.sot, st.lang_begin, st.n_languages, st.transcribe, st.translate,
                   st.notimestamps, list(gen.suppress_tokens) + [st.eot], gen.begin_suppress_tokens)
    with torch.no_grad():
        blang = m.detect_language(input_features=torch.from_numpy(bfeats)).numpy()
    m.generation_config.suppress_tokens = list(gen.suppress_tokens) + [st.eot]
    for j, w in enumerate(TURBO_BENCH_WINDOWS):
        # the seek loop's first pass (seek 0) is what bench.py decodes (max_passes=1); later passes are discarded
        with torch.no_grad():
            o = m.generate(torch.from_numpy(bfeats[j: j + 1]), task="transcribe", return_timestamps=True,
                           num_beams=1, max_new_tokens=128, return_segments=True)
        p = _passes_from_segments(o["segments"][0], 3)[0]
        a, b, c = _teacher_forced_pass_scores(m, bfeats[j], 0, [st.sot, int(blang[j]), st.transcribe], p, gb)
        res[f"bench_w{w}_lang"] = np.array([blang[j]], np.int32)
        res[f"bench_w{w}_tokens"] = np.array(p, np.int32)
        res[f"bench_w{w}_top_idx"], res[f"bench_w{w}_top_val"], res[f"bench_w{w}_ts_margin"] = a, b, c
    m.generation_config.suppress_tokens = list(gen.suppress_tokens)
    np.savez_compressed(os.path.join(out, "turbo.npz"), **res)


TURBO_BENCH_ALL = (0, 5, 11, 17, 22, 23)  # bench windows with an all-position golden (22, 23: the silent ones)


def _mask_intervals(mask: np.ndarray) -> np.ndarray:
    """[lo, hi) runs of True in a boolean row."""
    d = np.diff(np.concatenate([[0], mask.astype(np.int8), [0]]))
    return np.stack([np.flatnonzero(d == 1), np.flatnonzero(d == -1)], 1).astype(np.int32)


def make_turbo_bench(out):
    """bench.py's headline workload at every position: for TURBO_BENCH_ALL windows of workload(24, seed 1234), the
    fp32 first-pass decode (EOS suppressed, 128 new tokens, language detected), and along that sequence (teacher-
    forced) at each of the 128 positions: the raw logits' top-16 (indices, values, log-sum-exp), the processed top-16
    and the timestamp-rule margin, and the processors' -inf mask before the rule as [lo, hi) intervals. The mask plus
    the rule (tests/golden/turbo_parity.process_row) reproduces the oracle's process_logits exactly — asserted here on
    every fp32 row — so a device's raw logits can be processed on the host with the fp32 history (turbo_bench.npz)."""
    from transformers import WhisperFeatureExtractor
    from twamd.synth_audio import workload
    sys.path.insert(0, HERE)
    import turbo_parity as tp

    d = PRESETS["large-v3-turbo"]
    gen = GenerationSettings.default(d)
    st = gen.special
    sup = list(gen.suppress_tokens) + [st.eot]
    g = wo.GenCfg(d.vocab, st.eot, st.sot, st.lang_begin, st.n_languages, st.transcribe, st.translate,
                  st.notimestamps, sup, gen.begin_suppress_tokens)
    sd = wo.synth_state_dict(d.d_model, d.encoder_layers, d.decoder_layers, d.ffn, d.n_mels, d.vocab, SEED)
    m = hf_model(d, sd, gen)
    del sd
    fe = WhisperFeatureExtractor(feature_size=d.n_mels)
    wl = workload(24, 30.0, seed=1234)
    res = {"windows": np.array(TURBO_BENCH_ALL, np.int32)}
    m.generation_config.suppress_tokens = sup
    for w in TURBO_BENCH_ALL:
        feats = fe(wl[w], sampling_rate=16000, return_tensors="np")["input_features"][0]
        with torch.no_grad():
            lang = int(m.detect_language(input_features=torch.from_numpy(feats[None])).numpy()[0])
            o = m.generate(torch.from_numpy(feats[None]), task="transcribe", return_timestamps=True, num_beams=1,
                           max_new_tokens=128, return_segments=True)
        p = _passes_from_segments(o["segments"][0], 3)[0]
        assert len(p) == 128, len(p)
        prompt = [st.sot, lang, st.transcribe]
        ids = prompt + p[:-1]
        with torch.no_grad():
            lg = m(input_features=torch.from_numpy(feats[None]), decoder_input_ids=torch.tensor([ids])).logits[0].numpy()
        lg = lg[len(prompt) - 1:].astype(np.float32)
        assert lg.shape[0] == 128
        raw_i, raw_v, lse, pi, pv, mg, ivs, offs = [], [], [], [], [], [], [], [0]
        for t in range(128):
            row = lg[t]
            o16 = np.argsort(-row, kind="stable")[:16]
            raw_i.append(o16)
            raw_v.append(row[o16])
            mx = float(row.max())
            lse.append(mx + np.log(np.exp(row.astype(np.float64) - mx).sum()))
            ref = wo.process_logits(row, p[:t], g, True)
            iv = _mask_intervals(np.isneginf(wo.process_logits_no_rule(np.zeros_like(row), p[:t], g)))
            s, margin = tp.process_row(row, iv, st.timestamp_begin)
            assert np.array_equal(s, ref), (w, t)  # the host restatement of the chain is exact on the fp32 row
            assert int(np.argmax(ref)) == p[t], (w, t)  # generate() chose the processed argmax
            o16p = np.argsort(-ref, kind="stable")[:16]
            pi.append(o16p)
            pv.append(ref[o16p])
            mg.append(wo._ts_rule_margin(wo.process_logits_no_rule(row, p[:t], g), g.ts_begin))
            assert mg[-1] == margin or abs(mg[-1] - margin) < 1e-5, (w, t, mg[-1], margin)
            ivs.append(iv)
            offs.append(offs[-1] + len(iv))
        k = f"w{w}_"
        res[k + "lang"] = np.array([lang], np.int32)
        res[k + "tokens"] = np.array(p, np.int32)
        res[k + "raw_idx"], res[k + "raw_val"] = np.array(raw_i, np.int32), np.array(raw_v, np.float32)
        res[k + "lse"] = np.array(lse, np.float64)
        res[k + "top_idx"], res[k + "top_val"] = np.array(pi, np.int32), np.array(pv, np.float32)
        res[k + "ts_margin"] = np.array(mg, np.float32)
        res[k + "mask_iv"], res[k + "mask_off"] = np.concatenate(ivs), np.array(offs, np.int32)
        print(f"turbo_bench window {w}: lang {lang}, {len(p)} tokens, {sum(t >= st.timestamp_begin for t in p)} "
              f"timestamps", flush=True)
    m.generation_config.suppress_tokens = list(gen.suppress_tokens)
    np.savez_compressed(os.path.join(out, "turbo_bench.npz"), **res)


def make_turbo_beam(out):
    """large-v3-turbo, seeded synthetic weights: generate(num_beams=5) — the ASR pipeline's default decode
    (asr:160-163), i.e. what the reference's transcribe() runs — on TURBO_CLIPS, with timestamps (40 new tokens) and
    without (24). transformers' generate() gives the best hypothesis; the oracle's restatement of _beam_search
    (beam_search_core, pinned token-for-token to generate() at test-mini by test_oracle_golden.py), driven by the
    same fp32 model's logits, must return the same best hypothesis here too, and supplies all 5 finished hypotheses
    with their beam scores (sum of processed log-probs / generated length). A bf16 device decode may rank a near-tie
    the other way; the test accepts its hypothesis when it is one of these five and within a stated score tolerance
    of the best."""
    from transformers import WhisperFeatureExtractor
    from transformers.modeling_outputs import BaseModelOutput

    d = PRESETS["large-v3-turbo"]
    gen = GenerationSettings.default(d)
    st = gen.special
    sd = wo.synth_state_dict(d.d_model, d.encoder_layers, d.decoder_layers, d.ffn, d.n_mels, d.vocab, SEED)
    m = hf_model(d, sd, gen)
    del sd
    fe = WhisperFeatureExtractor(feature_size=d.n_mels)
    cl = clips()
    feats = np.stack([fe(cl[k], sampling_rate=16000, return_tensors="np")["input_features"][0] for k in TURBO_CLIPS])
    with torch.no_grad():
        lang = m.detect_language(input_features=torch.from_numpy(feats)).numpy()
        enc = m.model.encoder(torch.from_numpy(feats)).last_hidden_state
    res = {"lang": lang.astype(np.int32)}
    for ts, mnt in ((True, 40), (False, 24)):
        g = wo.GenCfg(d.vocab, st.eot, st.sot, st.lang_begin, st.n_languages, st.transcribe, st.translate,
                      st.notimestamps, gen.suppress_tokens, gen.begin_suppress_tokens)
        with torch.no_grad():
            hf = m.generate(torch.from_numpy(feats), task="transcribe", return_timestamps=ts, num_beams=5,
                            max_new_tokens=mnt, return_segments=True)
        tag = f"ts{int(ts)}"
        seqs, scores = [], []
        for i in range(len(TURBO_CLIPS)):
            prompt = [st.sot, int(lang[i]), st.transcribe] + ([] if ts else [st.notimestamps])
            e = BaseModelOutput(last_hidden_state=enc[i: i + 1])
            hist = {"h": [[] for _ in range(5)]}

            def logits_of(rows):
                ids = torch.tensor([prompt + r for r in rows])
                with torch.no_grad():
                    lg = m(encoder_outputs=BaseModelOutput(last_hidden_state=enc[i: i + 1].expand(len(rows), -1, -1)),
                           decoder_input_ids=ids).logits[:, -1].numpy()
                return [x.astype(np.float32) for x in lg]

            def step(srcs, toks):
                hist["h"] = [hist["h"][s_] + [t] for s_, t in zip(srcs, toks)]
                return logits_of(hist["h"])

            del e
            first = logits_of([[]])[0]
            best, tr = wo.beam_search_core(first, step, len(prompt), mnt, g, ts, 5)
            # generate()'s first seek pass (the whole window: the beams searched over features from seek 0)
            p0 = _passes_from_segments(hf["segments"][i], len(prompt))[0]
            ref = p0[: p0.index(st.eot) + 1] if st.eot in p0 else p0
            assert list(best) == ref, ("oracle beam search differs from generate()'s first pass", tag, i, best, ref)
            seqs.append([list(map(int, x)) for x in tr["fin_seq"]])
            scores.append(np.asarray(tr["fin_score"], np.float32))
        L = max(len(x) for c in seqs for x in c)
        arr = np.full((len(TURBO_CLIPS), 5, L), -1, np.int32)
        for i, c in enumerate(seqs):
            for k, x in enumerate(c):
                arr[i, k, : len(x)] = x
        res[f"{tag}_fin_seq"] = arr          # [clip][5][L], -1 padded, generated tokens incl. EOS
        res[f"{tag}_fin_score"] = np.stack(scores)
        res[f"{tag}_max_new_tokens"] = np.array([mnt], np.int32)
    np.savez_compressed(os.path.join(out, "turbo_beam.npz"), **res)


def make_turbo_word(out):
    """large-v3-turbo, seeded synthetic weights, the engine's default alignment heads (every head of the upper half
    of the decoder, GenerationSettings.default): generate(return_timestamps=True, return_token_timestamps=True,
    max_new_tokens=40) on TURBO_CLIPS — token-level timestamps from cross-attention DTW at the benchmarked depth."""
    from transformers import WhisperFeatureExtractor

    d = PRESETS["large-v3-turbo"]
    gen = GenerationSettings.default(d)
    sd = wo.synth_state_dict(d.d_model, d.encoder_layers, d.decoder_layers, d.ffn, d.n_mels, d.vocab, SEED)
    m = hf_model(d, sd, gen)
    del sd
    m.generation_config.alignment_heads = [list(h) for h in gen.alignment_heads]
    fe = WhisperFeatureExtractor(feature_size=d.n_mels)
    cl = clips()
    res = {}
    for i, name in enumerate(TURBO_CLIPS):
        f = fe(cl[name], sampling_rate=16000, return_tensors="pt", return_attention_mask=True)
        with torch.no_grad():
            o = m.generate(f["input_features"], attention_mask=f["attention_mask"], task="transcribe",
                           return_timestamps=True, return_token_timestamps=True, max_new_tokens=40)
        res[f"seq{i}"] = o["sequences"].numpy().astype(np.int32)
        res[f"ts{i}"] = o["token_timestamps"].numpy().astype(np.float32)
        res[f"nframes{i}"] = np.array([int(f["attention_mask"].sum())], np.int32)
    res["alignment_heads"] = np.array(gen.alignment_heads, np.int32)
    np.savez_compressed(os.path.join(out, "turbo_word.npz"), **res)


def make_large_v3(out):
    """openai/whisper-large-v3 dims — the reference's default model (vocalis/core/audio_pipeline.py:171): the turbo
    encoder with a 32-layer decoder — with the seeded synthetic weights, on clip speech30: encoder rows, teacher-forced
    raw logits over 24 positions, and generate(num_beams=1, return_timestamps=True, max_new_tokens=40) passes with
    their processed top-16 scores (transformers on CPU fp32)."""
    from transformers import WhisperFeatureExtractor

    d = PRESETS["large-v3"]
    gen = GenerationSettings.default(d)
    st = gen.special
    g = wo.GenCfg(d.vocab, st.eot, st.sot, st.lang_begin, st.n_languages, st.transcribe, st.translate,
                  st.notimestamps, gen.suppress_tokens, gen.begin_suppress_tokens)
    sd = wo.synth_state_dict(d.d_model, d.encoder_layers, d.decoder_layers, d.ffn, d.n_mels, d.vocab, SEED)
    m = hf_model(d, sd, gen)
    del sd
    fe = WhisperFeatureExtractor(feature_size=d.n_mels)
    feats = fe(clips()["speech30"], sampling_rate=16000, return_tensors="np")["input_features"]
    res = {}
    with torch.no_grad():
        enc = m.model.encoder(torch.from_numpy(feats)).last_hidden_state.numpy()
        lang = m.detect_language(input_features=torch.from_numpy(feats)).numpy()
        o = m.generate(torch.from_numpy(feats), task="transcribe", return_timestamps=True, num_beams=1,
                       max_new_tokens=40, return_segments=True)
    res["enc_rows_idx"] = np.array([0, 1, 750, 1499])
    res["enc_rows"] = enc[0, res["enc_rows_idx"]].astype(np.float32)
    res["lang"] = lang.astype(np.int32)
    res["gen_sequence"] = o["sequences"].numpy()[0].astype(np.int32)
    pr = [st.sot, int(lang[0]), st.transcribe]
    seek, ti, tv, mg, toks_all, seeks = 0, [], [], [], [], []
    for p in _passes_from_segments(o["segments"][0], 3):
        toks = p[: p.index(st.eot) + 1] if st.eot in p else p
        a, b, c = _teacher_forced_pass_scores(m, feats[0], seek, pr, toks, g)
        ti.append(a); tv.append(b); mg.append(c); toks_all.append(np.array(toks, np.int32)); seeks.append(seek)
        seq = toks[:-1] if toks and toks[-1] == st.eot else toks
        _, off = wo.retrieve_segment(seq, 3000 - seek, g.ts_begin)
        seek += off
    res["pass_len"] = np.array([len(x) for x in toks_all], np.int32)
    res["pass_seek"] = np.array(seeks, np.int32)
    res["pass_tokens"] = np.concatenate(toks_all)
    res["top_idx"], res["top_val"], res["ts_margin"] = np.concatenate(ti), np.concatenate(tv), np.concatenate(mg)
    p0 = pr + [int(t) for t in toks_all[0][:21]]
    res["tf_input_ids"] = np.array(p0[:24])
    with torch.no_grad():
        lg = m(input_features=torch.from_numpy(feats), decoder_input_ids=torch.tensor([p0[:24]])).logits[0].numpy()
    top = np.argsort(-lg, axis=1, kind="stable")[:, :16]
    res["tf_top_idx"] = top
    res["tf_top_val"] = np.take_along_axis(lg, top, 1).astype(np.float32)
    res["tf_lse"] = (np.log(np.exp(lg - lg.max(1, keepdims=True)).sum(1)) + lg.max(1)).astype(np.float64)
    res["sot_lang_logits"] = lg[0, st.lang_begin: st.lang_end].astype(np.float32)  # detect_language's candidates
    np.savez_compressed(os.path.join(out, "large_v3.npz"), **res)


def make_edge(out):
    """The ASR pipeline (test-mini, greedy, 8 new tokens, timestamps) on empty and sub-frame inputs, with the
    reference's chunking (60 / 5) and without: the output, or the exception type and message the reference's
    transcribe() would wrap as {"error": "Transcription error: <message>"}."""
    from transformers import AutomaticSpeechRecognitionPipeline, WhisperFeatureExtractor

    d = DIMS
    gen = GenerationSettings.default(d)
    sd = wo.synth_state_dict(d.d_model, d.encoder_layers, d.decoder_layers, d.ffn, d.n_mels, d.vocab, SEED)
    m = hf_model(d, sd, gen)
    fe = WhisperFeatureExtractor(feature_size=d.n_mels)
    pipe = AutomaticSpeechRecognitionPipeline(model=m, feature_extractor=fe, tokenizer=hf_tokenizer(gen.special),
                                              device=-1)
    cases = []
    for n in (0, 1, 160, 1600):
        for name, kw in (("ref_60_5", dict(chunk_length_s=60, stride_length_s=5, batch_size=32)), ("plain", {})):
            c = {"n_samples": n, "name": name, "kwargs": kw}
            try:
                c["output"] = _jsonable(pipe(np.zeros(n, np.float32), return_timestamps=True,
                                             generate_kwargs={"task": "transcribe", "num_beams": 1,
                                                              "max_new_tokens": 8}, **kw))
            except Exception as e:  # noqa: BLE001 - the reference's transcribe() catches everything
                c["error"] = {"type": type(e).__name__, "message": str(e)}
            cases.append(c)
    with open(os.path.join(out, "edge.json"), "w") as f:
        json.dump({"dims": "test-mini", "cases": cases}, f, indent=1)


def make_beam_long(out):
    """The reference's call (chunk_length_s=60, stride_length_s=5, batch_size=32, task only: the pipeline's default
    beam-5) on 8 minutes of audio at test-mini: 10 windows, so the drop-in's engine batch carries 50 beam rows."""
    from transformers import AutomaticSpeechRecognitionPipeline, WhisperFeatureExtractor

    d = DIMS
    gen = GenerationSettings.default(d)
    sd = wo.synth_state_dict(d.d_model, d.encoder_layers, d.decoder_layers, d.ffn, d.n_mels, d.vocab, SEED)
    m = hf_model(d, sd, gen)
    fe = WhisperFeatureExtractor(feature_size=d.n_mels)
    pipe = AutomaticSpeechRecognitionPipeline(model=m, feature_extractor=fe, tokenizer=hf_tokenizer(gen.special),
                                              device=-1)
    audio = np.concatenate([speech_like(200.0, 21), white_noise(80.0, 22), speech_like(200.0, 23)])  # 480 s
    kw = dict(chunk_length_s=60, stride_length_s=5, batch_size=32)
    r = pipe(audio.copy(), generate_kwargs={"task": "transcribe", "max_new_tokens": 24}, return_timestamps=True, **kw)
    with open(os.path.join(out, "beam_long.json"), "w") as f:
        json.dump({"dims": "test-mini", "audio": "speech_like(200,21)+white_noise(80,22)+speech_like(200,23)",
                   "kwargs": kw, "max_new_tokens": 24, "output": _jsonable(r)}, f)


def make_options(out):
    """The ASR pipeline at test-mini on 75 s of audio with the call options a user of the reference's transcribe()
    can reach: task="translate" with the reference's call (default beam-5), return_timestamps=False, a forced
    language, return_language=True (greedy where not the reference's call)."""
    from transformers import AutomaticSpeechRecognitionPipeline, WhisperFeatureExtractor

    d = DIMS
    gen = GenerationSettings.default(d)
    sd = wo.synth_state_dict(d.d_model, d.encoder_layers, d.decoder_layers, d.ffn, d.n_mels, d.vocab, SEED)
    m = hf_model(d, sd, gen)
    fe = WhisperFeatureExtractor(feature_size=d.n_mels)
    pipe = AutomaticSpeechRecognitionPipeline(model=m, feature_extractor=fe, tokenizer=hf_tokenizer(gen.special),
                                              device=-1)
    audio = np.concatenate([speech_like(40.0, 5), white_noise(35.0, 11)])
    ref = dict(chunk_length_s=60, stride_length_s=5, batch_size=32)
    cases = [
        ("translate_ref_call", ref, {"task": "translate", "max_new_tokens": 24}, True, {}),
        ("translate_greedy", ref, {"task": "translate", "num_beams": 1, "max_new_tokens": 24}, True, {}),
        ("no_timestamps", dict(chunk_length_s=30, stride_length_s=0, batch_size=2),
         {"task": "transcribe", "num_beams": 1, "max_new_tokens": 24}, False, {}),
        ("language_fr", ref, {"task": "transcribe", "language": "fr", "num_beams": 1, "max_new_tokens": 24}, True, {}),
        ("return_language", ref, {"task": "transcribe", "num_beams": 1, "max_new_tokens": 24}, True,
         {"return_language": True}),
    ]
    res = []
    for name, kw, gk, ts, extra in cases:
        c = {"name": name, "kwargs": kw, "generate_kwargs": gk, "return_timestamps": ts, "extra": extra}
        try:
            c["output"] = _jsonable(pipe(audio.copy(), generate_kwargs=dict(gk), return_timestamps=ts, **kw, **extra))
        except Exception as e:  # noqa: BLE001 - recorded as the reference would surface it
            c["error"] = {"type": type(e).__name__, "message": str(e)}
        res.append(c)
    with open(os.path.join(out, "options.json"), "w") as f:
        json.dump({"dims": "test-mini", "audio": "speech_like(40,5)+white_noise(35,11)", "cases": res}, f, indent=1)


SWEEP_CASES = [  # name, audio [(kind, seconds, seed)], pipeline kwargs, generate_kwargs, return_timestamps
    ("c20_s4_greedy", [("speech", 50.0, 31), ("noise", 20.0, 32)], dict(chunk_length_s=20, stride_length_s=4, batch_size=3),
     {"task": "transcribe", "num_beams": 1, "max_new_tokens": 32}, True),
    ("c45_asym_beam3", [("speech", 70.0, 33)], dict(chunk_length_s=45, stride_length_s=(6, 3), batch_size=4),
     {"task": "transcribe", "num_beams": 3, "max_new_tokens": 20}, True),
    ("c30_greedy_nots", [("noise", 30.0, 34), ("speech", 40.0, 35)], dict(chunk_length_s=30, stride_length_s=0, batch_size=5),
     {"task": "transcribe", "num_beams": 1, "max_new_tokens": 40}, False),
    ("nochunk_beam5", [("speech", 25.0, 36)], {}, {"task": "transcribe", "num_beams": 5, "max_new_tokens": 24}, True),
    ("c15_translate_greedy", [("speech", 60.0, 37), ("silence", 10.0, 0)],
     dict(chunk_length_s=15, stride_length_s=3, batch_size=8), {"task": "translate", "num_beams": 1, "max_new_tokens": 24},
     True),
    ("c10_greedy", [("speech", 100.0, 38)], dict(chunk_length_s=10, stride_length_s=2, batch_size=16),
     {"task": "transcribe", "num_beams": 1, "max_new_tokens": 16}, True),
    ("ref_de_beam5", [("speech", 180.0, 39)], dict(chunk_length_s=60, stride_length_s=5, batch_size=32),
     {"task": "transcribe", "language": "de", "max_new_tokens": 24}, True),
]


def sweep_audio(spec):
    parts = []
    for kind, sec, seed in spec:
        parts.append(speech_like(sec, seed) if kind == "speech" else white_noise(sec, seed) if kind == "noise"
                     else silence(sec))
    return np.concatenate(parts).astype(np.float32)


def make_sweep(out):
    """The ASR pipeline at test-mini over a sweep of chunk / stride / batch sizes, greedy and beam, timestamps on and
    off, translate and a forced language (SWEEP_CASES): outputs for the engine's end-to-end comparison."""
    from transformers import AutomaticSpeechRecognitionPipeline, WhisperFeatureExtractor

    d = DIMS
    gen = GenerationSettings.default(d)
    sd = wo.synth_state_dict(d.d_model, d.encoder_layers, d.decoder_layers, d.ffn, d.n_mels, d.vocab, SEED)
    m = hf_model(d, sd, gen)
    fe = WhisperFeatureExtractor(feature_size=d.n_mels)
    pipe = AutomaticSpeechRecognitionPipeline(model=m, feature_extractor=fe, tokenizer=hf_tokenizer(gen.special),
                                              device=-1)
    res = []
    for name, spec, kw, gk, ts in SWEEP_CASES:
        r = pipe(sweep_audio(spec), generate_kwargs=dict(gk), return_timestamps=ts, **kw)
        res.append({"name": name, "audio": spec, "kwargs": kw, "generate_kwargs": gk, "return_timestamps": ts,
                    "output": _jsonable(r)})
    with open(os.path.join(out, "sweep.json"), "w") as f:
        json.dump({"dims": "test-mini", "cases": res}, f, indent=1)


LONGFORM_CASES = [  # name, pipeline kwargs, generate_kwargs, return_timestamps
    ("long_greedy", {}, {"task": "transcribe", "num_beams": 1, "max_new_tokens": 40}, True),
    ("long_beam3", {}, {"task": "transcribe", "num_beams": 3, "max_new_tokens": 24}, True),
    ("long_cond", {}, {"task": "transcribe", "num_beams": 1, "max_new_tokens": 40, "condition_on_prev_tokens": True},
     True),
    ("long_no_ts", {}, {"task": "transcribe", "num_beams": 1, "max_new_tokens": 40}, False),
    ("chunk30_cond_b3", dict(chunk_length_s=30, stride_length_s=0, batch_size=3),
     {"task": "transcribe", "num_beams": 1, "max_new_tokens": 40, "condition_on_prev_tokens": True}, True),
]


def make_longform(out):
    """Long-form input (75 s, no chunk_length_s: generate()'s sequential seek loop over the features of the whole
    input, asr:450-457) and condition_on_prev_tokens at test-mini: the pipeline outputs (or the error it raises), the
    long-form features of the feature extractor (truncation=False, padding="longest"), and per case every seek pass's
    decoder prompt and raw output as generate_with_fallback saw them (a spy: conditioning prompts are built from the
    previous passes' segments, generation_whisper.py:1853-1918)."""
    from transformers import AutomaticSpeechRecognitionPipeline, WhisperFeatureExtractor
    from transformers.models.whisper import generation_whisper as gw

    d = DIMS
    gen = GenerationSettings.default(d)
    sd = wo.synth_state_dict(d.d_model, d.encoder_layers, d.decoder_layers, d.ffn, d.n_mels, d.vocab, SEED)
    m = hf_model(d, sd, gen)
    fe = WhisperFeatureExtractor(feature_size=d.n_mels)
    pipe = AutomaticSpeechRecognitionPipeline(model=m, feature_extractor=fe, tokenizer=hf_tokenizer(gen.special),
                                              device=-1)
    audio = np.concatenate([speech_like(40.0, 5), white_noise(35.0, 11)]).astype(np.float32)
    f = fe(audio, sampling_rate=16000, truncation=False, padding="longest", return_tensors="np")["input_features"][0]
    feats = {"shape": list(f.shape), "sub": f[:, ::97].tolist(), "colsum": f.sum(axis=0)[::7].tolist()}
    orig = gw.WhisperGenerationMixin.generate_with_fallback
    log = []

    def spy(self, *a, **kw):
        r = orig(self, *a, **kw)
        log.append({"prompts": kw["decoder_input_ids"].tolist(), "rows": [int(i) for i in kw["batch_idx_map"]],
                    "seek": kw["seek"].tolist(), "sequences": [x.tolist() for x in r[0]]})
        return r

    res = []
    gw.WhisperGenerationMixin.generate_with_fallback = spy
    try:
        for name, kw, gk, ts in LONGFORM_CASES:
            log.clear()
            c = {"name": name, "kwargs": kw, "generate_kwargs": gk, "return_timestamps": ts}
            try:
                c["output"] = _jsonable(pipe(audio.copy(), generate_kwargs=dict(gk), return_timestamps=ts, **kw))
            except Exception as e:  # noqa: BLE001 - recorded as the reference would surface it
                c["error"] = {"type": type(e).__name__, "message": str(e)}
            c["passes"] = list(log)
            res.append(c)
    finally:
        gw.WhisperGenerationMixin.generate_with_fallback = orig
    with open(os.path.join(out, "longform.json"), "w") as fo:
        json.dump({"dims": "test-mini", "audio": "speech_like(40,5)+white_noise(35,11)", "n_samples": len(audio),
                   "features": feats, "cases": res}, fo)


PROMPT_TOKENS = [1000, 2000, 3000, 4000, 5000, 6000]  # the prompt's text tokens (prompt_ids = [<|startofprev|>] + these)
PROMPT_CASES = [  # name, pipeline kwargs, generate_kwargs (prompt_ids added by the maker), return_timestamps
    ("chunk30_prompt_b3", dict(chunk_length_s=30, stride_length_s=0, batch_size=3),
     {"task": "transcribe", "num_beams": 1, "max_new_tokens": 40}, True),
    ("long_prompt", {}, {"task": "transcribe", "num_beams": 1, "max_new_tokens": 40}, True),
    ("long_prompt_cond", {}, {"task": "transcribe", "num_beams": 1, "max_new_tokens": 40,
                              "condition_on_prev_tokens": True}, True),
    ("long_prompt_all", {}, {"task": "transcribe", "num_beams": 1, "max_new_tokens": 40,
                             "condition_on_prev_tokens": True, "prompt_condition_type": "all-segments"}, True),
    ("chunk30_prompt_no_ts", dict(chunk_length_s=30, stride_length_s=0, batch_size=3),
     {"task": "transcribe", "num_beams": 1, "max_new_tokens": 40}, False),
]


def make_prompt(out):
    """prompt_ids (generate()'s initial prompt, generation_whisper.py:1119-1124, 1885-1912) at test-mini on the 75-s
    audio of make_longform: chunked 30-s windows and long-form, with and without condition_on_prev_tokens, both
    prompt_condition_type values; the pipeline outputs and every seek pass's decoder prompt and raw output (the same
    spy as make_longform)."""
    from transformers import AutomaticSpeechRecognitionPipeline, WhisperFeatureExtractor
    from transformers.models.whisper import generation_whisper as gw

    d = DIMS
    gen = GenerationSettings.default(d)
    sd = wo.synth_state_dict(d.d_model, d.encoder_layers, d.decoder_layers, d.ffn, d.n_mels, d.vocab, SEED)
    m = hf_model(d, sd, gen)
    fe = WhisperFeatureExtractor(feature_size=d.n_mels)
    pipe = AutomaticSpeechRecognitionPipeline(model=m, feature_extractor=fe, tokenizer=hf_tokenizer(gen.special),
                                              device=-1)
    audio = np.concatenate([speech_like(40.0, 5), white_noise(35.0, 11)]).astype(np.float32)
    # <|startofprev|>: a real checkpoint's generation_config names it (prev_sot_token_id); this synthetic one gets the
    # token transformers falls back to without it (suppress_tokens[-2], generation_whisper.py:1876-1881)
    m.generation_config.prev_sot_token_id = int(m.generation_config.suppress_tokens[-2])
    prompt = [int(m.generation_config.prev_sot_token_id)] + PROMPT_TOKENS
    orig = gw.WhisperGenerationMixin.generate_with_fallback
    log = []

    def spy(self, *a, **kw):
        r = orig(self, *a, **kw)
        log.append({"prompts": kw["decoder_input_ids"].tolist(), "rows": [int(i) for i in kw["batch_idx_map"]],
                    "seek": kw["seek"].tolist(), "sequences": [x.tolist() for x in r[0]]})
        return r

    res = []
    gw.WhisperGenerationMixin.generate_with_fallback = spy
    try:
        for name, kw, gk, ts in PROMPT_CASES:
            log.clear()
            c = {"name": name, "kwargs": kw, "generate_kwargs": gk, "return_timestamps": ts}
            try:
                c["output"] = _jsonable(pipe(audio.copy(), generate_kwargs=dict(gk, prompt_ids=torch.tensor(prompt)),
                                             return_timestamps=ts, **kw))
            except Exception as e:  # noqa: BLE001 - recorded as the reference would surface it
                c["error"] = {"type": type(e).__name__, "message": str(e)}
            c["passes"] = list(log)
            res.append(c)
    finally:
        gw.WhisperGenerationMixin.generate_with_fallback = orig
    with open(os.path.join(out, "prompt.json"), "w") as fo:
        json.dump({"dims": "test-mini", "audio": "speech_like(40,5)+white_noise(35,11)", "prompt_ids": prompt,
                   "cases": res}, fo)


TINY_CLIPS = ("speech30", "noise12")


def make_tiny(out):
    """whisper-tiny.en dims (BASELINE configs[0]: d 384, 4 + 4 layers, 6 heads, 80 mels, English-only vocabulary
    51864) with the seeded synthetic weights: encoder output rows, teacher-forced logits along clip 0's first pass
    and generate() (no language / task tokens: the English-only prompt is <|startoftranscript|> alone) with the
    processed top-16 scores of every pass, from transformers on CPU fp32. Pins the oracle at tiny.en
    (tests/test_oracle_golden.py) and the engine on the GPU (tests/test_gpu_configs.py)."""
    from transformers import WhisperFeatureExtractor

    d = PRESETS["tiny.en"]
    gen = GenerationSettings.default(d)
    st = gen.special
    assert not st.is_multilingual
    g = wo.GenCfg(d.vocab, st.eot, st.sot, st.lang_begin, st.n_languages, st.transcribe, st.translate,
                  st.notimestamps, gen.suppress_tokens, gen.begin_suppress_tokens, multilingual=False)
    sd = wo.synth_state_dict(d.d_model, d.encoder_layers, d.decoder_layers, d.ffn, d.n_mels, d.vocab, SEED)
    m = hf_model(d, sd, gen)
    # an English-only checkpoint's generation_config has no language / task tables (generate() would otherwise run
    # language detection: generation_whisper.py _retrieve_init_tokens)
    delattr(m.generation_config, "lang_to_id")
    delattr(m.generation_config, "task_to_id")
    fe = WhisperFeatureExtractor(feature_size=d.n_mels)
    cl = clips()
    feats = np.stack([fe(cl[k], sampling_rate=16000, return_tensors="np")["input_features"][0] for k in TINY_CLIPS])
    res = {}
    with torch.no_grad():
        enc = m.model.encoder(torch.from_numpy(feats)).last_hidden_state.numpy()
    res["enc_rows_idx"] = np.array([0, 1, 2, 375, 750, 1124, 1498, 1499])
    res["enc_rows"] = enc[:, res["enc_rows_idx"]].astype(np.float32)
    res["enc_mean"] = enc.mean(axis=(1, 2))
    res["enc_std"] = enc.std(axis=(1, 2))
    res["enc_row_norm"] = np.linalg.norm(enc, axis=2).astype(np.float32)
    with torch.no_grad():
        o = m.generate(torch.from_numpy(feats), return_timestamps=True, num_beams=1, max_new_tokens=48,
                       return_segments=True)
    res["gen_sequences"] = o["sequences"].numpy()
    pr = [st.sot]
    for i in range(len(TINY_CLIPS)):
        passes = _passes_from_segments(o["segments"][i], len(pr))
        seek, ti, tv, mg, kept, offs = 0, [], [], [], [], [0]
        for q in passes:
            toks = q[: q.index(st.eot) + 1] if st.eot in q else q
            a, b, c = _teacher_forced_pass_scores(m, feats[i], seek, pr, toks, g)
            ti.append(a); tv.append(b); mg.append(c)
            seq = toks[:-1] if toks and toks[-1] == st.eot else toks
            seg, off = wo.retrieve_segment(seq, 3000 - seek, g.ts_begin)
            kept += seg
            seek += off
            offs.append(seek)
        ref = [int(t) for t in res["gen_sequences"][i]]
        while ref and ref[-1] == st.eot:
            ref.pop()
        assert kept == ref, ("pass reconstruction differs from generate()", i)
        res[f"gen{i}_pass_len"] = np.array([len(x) for x in ti], np.int32)
        res[f"gen{i}_pass_tokens"] = np.concatenate(
            [np.array(q[: len(x)], np.int32) for q, x in zip(passes, ti)]) if passes else np.zeros(0, np.int32)
        res[f"gen{i}_pass_seek"] = np.array(offs[:-1], np.int32)
        res[f"gen{i}_top_idx"], res[f"gen{i}_top_val"] = np.concatenate(ti), np.concatenate(tv)
        res[f"gen{i}_ts_margin"] = np.concatenate(mg)
    p0 = pr + [int(t) for t in res["gen0_pass_tokens"][:23]]
    res["tf_input_ids"] = np.array(p0[:24])
    with torch.no_grad():
        lg = m(input_features=torch.from_numpy(feats[:1]), decoder_input_ids=torch.tensor([p0[:24]])).logits[0].numpy()
    top = np.argsort(-lg, axis=1, kind="stable")[:, :16]
    res["tf_top_idx"] = top
    res["tf_top_val"] = np.take_along_axis(lg, top, 1).astype(np.float32)
    res["tf_lse"] = (np.log(np.exp(lg - lg.max(1, keepdims=True)).sum(1)) + lg.max(1)).astype(np.float64)
    np.savez_compressed(os.path.join(out, "tiny.npz"), **res)


FALLBACK_CLIPS = ("speech30", "noise12", "zeros30")
FALLBACK_SKIP = {"temperature": [0.0], "compression_ratio_threshold": None, "logprob_threshold": -3.0,
                 "no_speech_threshold": 3e-5}


def make_fallback(out):
    """generate()'s temperature-fallback criteria on test-mini (generation_whisper.py:970-1116, 1243-1287): every
    _need_fallback call is spied on (its seek_sequence, transformers' own _retrieve_compression_ratio and
    _retrieve_avg_logprobs on it, WhisperNoSpeechDetection's no_speech_prob, and the returned decision) in
      "metrics": inert thresholds (nothing fires; every pass's criteria are recorded), temperature (0.0,);
      "skip":    FALLBACK_SKIP (the silent window's first pass has avg logprob < -3 and no_speech_prob > 3e-5: it is
                 skipped; the others keep their greedy tokens), temperature (0.0,) — a deterministic outcome,
    with the final generate() sequences of both. Sampled retries (temperature > 0) draw from torch's random stream and
    are not fixtures."""
    from transformers import WhisperFeatureExtractor
    from transformers.generation.logits_process import WhisperNoSpeechDetection
    from transformers.models.whisper.generation_whisper import _get_attr_from_logit_processors

    d = DIMS
    gen = GenerationSettings.default(d)
    sd = wo.synth_state_dict(d.d_model, d.encoder_layers, d.decoder_layers, d.ffn, d.n_mels, d.vocab, SEED)
    fe = WhisperFeatureExtractor(feature_size=d.n_mels)
    cl = clips()
    feats = torch.from_numpy(np.stack([fe(cl[k], sampling_rate=16000, return_tensors="np")["input_features"][0]
                                       for k in FALLBACK_CLIPS]))
    res = {"seed": SEED, "dims": "test-mini", "clips": list(FALLBACK_CLIPS), "max_new_tokens": 40}
    for name, kw in (("metrics", {"temperature": [0.0], "compression_ratio_threshold": 1e9, "logprob_threshold": -1e9,
                                  "no_speech_threshold": 2.0}),
                     ("skip", FALLBACK_SKIP)):
        m = hf_model(d, sd, gen)
        rec = []
        orig = m._need_fallback

        def spy(seek_sequence, seek_outputs, index, logits_processor, generation_config, vocab_size, temperature,
                _m=m, _orig=orig, _rec=rec):
            cr = _m._retrieve_compression_ratio(seek_sequence, vocab_size)
            lp = _m._retrieve_avg_logprobs(seek_outputs[index]["scores"], seek_sequence, temperature)
            nsp = _get_attr_from_logit_processors(logits_processor, WhisperNoSpeechDetection, "no_speech_prob")
            o = _orig(seek_sequence, seek_outputs, index, logits_processor, generation_config, vocab_size, temperature)
            _rec.append({"index": int(index), "tokens": [int(t) for t in seek_sequence.tolist()],
                         "compression_ratio": float(cr), "avg_logprob": float(lp),
                         "no_speech_prob": None if nsp is None else float(nsp[index]),
                         "needs_fallback": bool(o[0]), "should_skip": bool(o[1])})
            return o

        m._need_fallback = spy
        with torch.no_grad():
            o = m.generate(feats, task="transcribe", return_timestamps=True, max_new_tokens=40, return_segments=True,
                           temperature=tuple(kw["temperature"]),
                           **{k: v for k, v in kw.items() if k != "temperature" and v is not None})
        res[name] = {"kwargs": kw, "calls": rec, "sequences": o["sequences"].tolist()}
    with open(os.path.join(out, "fallback.json"), "w") as f:
        json.dump(res, f)


def make_fallback_beam(out):
    """The temperature fallback with beam search (num_beams=3; generate_with_fallback, generation_whisper.py:970-1116):
    spied like make_fallback. The beam pass's average log-probability is _retrieve_avg_logprobs over the processed
    beam scores gathered along the hypothesis' beam_indices (log_softmax renormalises them over the allowed tokens);
    "metrics": inert thresholds, every pass's criteria; "skip": FALLBACK_SKIP with beams; "resample": temperature
    (0.0, 0.4) with logprob_threshold -2.5: the calls record the decoding mode (a sampling round sets
    generation_config.num_beams = 1 for the rest of the generate() call) and the first round's decisions."""
    from transformers import WhisperFeatureExtractor
    from transformers.generation.logits_process import WhisperNoSpeechDetection
    from transformers.models.whisper.generation_whisper import _get_attr_from_logit_processors

    d = DIMS
    gen = GenerationSettings.default(d)
    sd = wo.synth_state_dict(d.d_model, d.encoder_layers, d.decoder_layers, d.ffn, d.n_mels, d.vocab, SEED)
    fe = WhisperFeatureExtractor(feature_size=d.n_mels)
    cl = clips()
    feats = torch.from_numpy(np.stack([fe(cl[k], sampling_rate=16000, return_tensors="np")["input_features"][0]
                                       for k in FALLBACK_CLIPS]))
    res = {"seed": SEED, "dims": "test-mini", "clips": list(FALLBACK_CLIPS), "max_new_tokens": 24, "num_beams": 3}
    for name, kw in (("metrics", {"temperature": [0.0], "compression_ratio_threshold": 1e9, "logprob_threshold": -1e9,
                                  "no_speech_threshold": 2.0}),
                     ("skip", FALLBACK_SKIP),
                     ("resample", {"temperature": [0.0, 0.4], "compression_ratio_threshold": None,
                                   "logprob_threshold": -2.5, "no_speech_threshold": None})):
        m = hf_model(d, sd, gen)
        rec = []
        orig = m._need_fallback

        def spy(seek_sequence, seek_outputs, index, logits_processor, generation_config, vocab_size, temperature,
                _m=m, _orig=orig, _rec=rec):
            cr = _m._retrieve_compression_ratio(seek_sequence, vocab_size)
            lp = _m._retrieve_avg_logprobs(seek_outputs[index]["scores"], seek_sequence, temperature)
            nsp = _get_attr_from_logit_processors(logits_processor, WhisperNoSpeechDetection, "no_speech_prob")
            o = _orig(seek_sequence, seek_outputs, index, logits_processor, generation_config, vocab_size, temperature)
            _rec.append({"index": int(index), "tokens": [int(t) for t in seek_sequence.tolist()],
                         "temperature": temperature, "num_beams": int(generation_config.num_beams),
                         "compression_ratio": float(cr), "avg_logprob": float(lp),
                         "no_speech_prob": None if nsp is None else float(nsp[index]),
                         "needs_fallback": bool(o[0]), "should_skip": bool(o[1])})
            return o

        m._need_fallback = spy
        torch.manual_seed(0)
        with torch.no_grad():
            o = m.generate(feats, task="transcribe", return_timestamps=True, max_new_tokens=24, return_segments=True,
                           num_beams=3, temperature=tuple(kw["temperature"]),
                           **{k: v for k, v in kw.items() if k != "temperature" and v is not None})
        res[name] = {"kwargs": kw, "calls": rec, "sequences": o["sequences"].tolist()}
    with open(os.path.join(out, "fallback_beam.json"), "w") as f:
        json.dump(res, f)


def _jsonable(x):
    if isinstance(x, dict):
        return {k: _jsonable(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_jsonable(v) for v in x]
    if isinstance(x, (np.floating, np.integer)):
        return x.item()
    return x


if __name__ == "__main__":
    torch.manual_seed(0)
    torch.set_num_threads(max(1, os.cpu_count() or 1))
    which = sys.argv[1:] or ["logmel", "model", "pipeline", "decode_asr"]
    for w in which:
        globals()[f"make_{w}"](HERE)
        print("wrote", w)

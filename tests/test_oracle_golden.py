"""Pin the CPU oracle (oracle/whisper_oracle.py) against golden vectors produced by transformers itself
(tests/golden/make_golden.py, same seeded weights). CPU only."""
import os

import numpy as np
import pytest

from oracle import whisper_oracle as wo
from twamd.config import PRESETS, GenerationSettings
from twamd.synth_audio import silence, speech_like, white_noise

G = os.path.join(os.path.dirname(__file__), "golden")
D = PRESETS["test-mini"]


def _clips():
    return {"speech30": speech_like(30.0, 1234), "noise12": white_noise(12.3, 7), "zeros30": silence(30.0),
            "speech45": speech_like(45.0, 99)}


@pytest.fixture(scope="module")
def golden_model():
    return np.load(os.path.join(G, "model.npz"))


@pytest.fixture(scope="module")
def oracle_model():
    sd = wo.synth_state_dict(D.d_model, D.encoder_layers, D.decoder_layers, D.ffn, D.n_mels, D.vocab, 1234)
    return wo.WhisperOracle(sd, D.heads)


@pytest.fixture(scope="module")
def gcfg():
    gen = GenerationSettings.default(D)
    st = gen.special
    return wo.GenCfg(D.vocab, st.eot, st.sot, st.lang_begin, st.n_languages, st.transcribe, st.translate,
                     st.notimestamps, gen.suppress_tokens, gen.begin_suppress_tokens)


def test_synth_uniform_is_bf16_exact_and_bounded():
    v = wo.synth_uniform(1234, 77, 100000, 0.05, 0.0)
    assert np.all(np.abs(v) <= 0.05 * (1 + 2 ** -8))  # bf16 rounding may step just past the scale
    assert np.all((v.view(np.uint32) & 0xFFFF) == 0)      # bf16-representable
    assert abs(float(v.std()) - 0.05 / np.sqrt(3)) < 1e-3
    assert not np.array_equal(v, wo.synth_uniform(1235, 77, 100000, 0.05, 0.0))


@pytest.mark.parametrize("n_mels,name", [(128, "speech30"), (128, "noise12"), (128, "zeros30"), (128, "speech45"),
                                         (80, "speech30")])
def test_logmel_matches_feature_extractor(n_mels, name):
    g = np.load(os.path.join(G, "logmel.npz"))
    f = wo.log_mel(_clips()[name], n_mels)
    assert f.shape == (n_mels, 3000)
    np.testing.assert_allclose(f[:, ::15], g[f"feat{n_mels}_{name}_sub"], atol=2e-5, rtol=0)
    np.testing.assert_allclose(f.sum(axis=1), g[f"feat{n_mels}_{name}_rowsum"], rtol=1e-5, atol=1e-3)


def test_encoder_matches_transformers(golden_model, oracle_model):
    feats = wo.log_mel(speech_like(30.0, 1234), 128)
    enc = oracle_model.encode(feats)
    np.testing.assert_allclose(enc[golden_model["enc_rows_idx"]], golden_model["enc_rows"][0], atol=2e-3, rtol=0)
    assert abs(enc.mean() - golden_model["enc_mean"][0]) < 1e-4
    assert abs(enc.std() - golden_model["enc_std"][0]) < 1e-4


def test_teacher_forced_logits_match(golden_model, oracle_model):
    feats = wo.log_mel(speech_like(30.0, 1234), 128)
    enc = oracle_model.encode(feats)
    cache = oracle_model.new_cache(enc)
    ids = golden_model["tf_input_ids"]
    for t, tok in enumerate(ids):
        lg = oracle_model.decoder_step(int(tok), cache)
        top = golden_model["tf_top_idx"][t]
        np.testing.assert_allclose(lg[top], golden_model["tf_top_val"][t], atol=2e-3)
        assert int(np.argmax(lg)) == int(top[0])
        m = lg.max()
        assert abs(float(m + np.log(np.exp(lg - m).sum())) - golden_model["tf_lse"][t]) < 2e-3


def test_language_detection_and_generate_match(golden_model, oracle_model, gcfg):
    clips = _clips()
    for i, name in enumerate(("speech30", "noise12")):
        feats = wo.log_mel(clips[name], 128)
        toks, lang = wo.generate(oracle_model, feats, gcfg, task="transcribe", return_timestamps=True,
                                 max_new_tokens=40)
        assert lang == int(golden_model["gen_lang"][i])
        ref = [int(t) for t in golden_model["gen_sequences"][i]]
        while ref and ref[-1] == gcfg.eot:
            ref.pop()
        assert toks == ref, (name, toks, ref)


@pytest.mark.parametrize("case", [0, 1, 2])
def test_beam_search_matches_transformers(oracle_model, gcfg, case):
    """The oracle's restatement of _beam_search (num_beams=5, the ASR pipeline's default) reproduces
    transformers' generate() token-for-token (tests/golden/beam.json)."""
    import json

    gold = json.load(open(os.path.join(G, "beam.json")))
    c = gold["cases"][case]
    cl = _clips()
    for name, ref in zip(c["clips"], c["sequences"]):
        feats = wo.log_mel(cl[name][:480000], D.n_mels)
        got, _ = wo.generate(oracle_model, feats, gcfg, task="transcribe", return_timestamps=c["return_timestamps"],
                             max_new_tokens=c["max_new_tokens"], num_beams=gold["num_beams"])
        while ref and ref[-1] == gcfg.eot:
            ref = ref[:-1]
        assert got == ref, (name, got[:20], ref[:20])


def test_dtw_and_median_filter_match_transformers():
    z = np.load(os.path.join(G, "word.npz"))
    for k in range(4):
        ti, tj = wo.dynamic_time_warping(z[f"dtw{k}_in"])
        assert np.array_equal(ti, z[f"dtw{k}_text"]) and np.array_equal(tj, z[f"dtw{k}_time"])
    np.testing.assert_array_equal(wo.median_filter(z["median_in"], 7), z["median_out"])


@pytest.mark.parametrize("name", ["speech30", "noise12"])
def test_token_timestamps_match_transformers(oracle_model, gcfg, name):
    """generate(return_token_timestamps=True): cross-attention of the alignment heads -> normalise -> median filter
    -> DTW, per seek pass (tests/golden/word.npz)."""
    z = np.load(os.path.join(G, "word.npz"))
    x = _clips()[name]
    feats = wo.log_mel(x[:480000], D.n_mels)
    nf = min(480000, len(x)) // 160 + (1 if min(480000, len(x)) % 160 else 0)
    toks, _, tts, _ = wo.generate(oracle_model, feats, gcfg, task="transcribe", return_timestamps=True,
                                  max_new_tokens=40, alignment_heads=[(1, 0), (1, 1), (1, 2), (1, 3)], num_frames=nf)
    assert toks == z[f"gen_{name}_seq"][0].tolist()
    np.testing.assert_allclose(tts, z[f"gen_{name}_ts"][0], atol=1e-6)


# ---- whisper-tiny.en (BASELINE configs[0]): English-only vocabulary, 80 mels, no language / task tokens ----------
TINY = PRESETS["tiny.en"]


@pytest.fixture(scope="module")
def tiny_golden():
    return np.load(os.path.join(G, "tiny.npz"))


@pytest.fixture(scope="module")
def tiny_oracle():
    d = TINY
    return wo.WhisperOracle(wo.synth_state_dict(d.d_model, d.encoder_layers, d.decoder_layers, d.ffn, d.n_mels,
                                                d.vocab, 1234), d.heads)


def test_tiny_en_encoder_and_logits_match_transformers(tiny_golden, tiny_oracle):
    z = tiny_golden
    enc = tiny_oracle.encode(wo.log_mel(speech_like(30.0, 1234), TINY.n_mels))
    np.testing.assert_allclose(enc[z["enc_rows_idx"]], z["enc_rows"][0], atol=2e-3, rtol=0)
    assert abs(enc.mean() - z["enc_mean"][0]) < 1e-4 and abs(enc.std() - z["enc_std"][0]) < 1e-4
    cache = tiny_oracle.new_cache(enc)
    for t, tok in enumerate(z["tf_input_ids"]):
        lg = tiny_oracle.decoder_step(int(tok), cache)
        top = z["tf_top_idx"][t]
        np.testing.assert_allclose(lg[top], z["tf_top_val"][t], atol=2e-3)
        m = lg.max()
        assert abs(float(m + np.log(np.exp(lg - m).sum())) - z["tf_lse"][t]) < 2e-3


def test_tiny_en_generate_matches_transformers(tiny_golden, tiny_oracle):
    """English-only generate(): prompt <|startoftranscript|> alone (no detection, no task), seek loop included."""
    gen = GenerationSettings.default(TINY)
    st = gen.special
    g = wo.GenCfg(TINY.vocab, st.eot, st.sot, st.lang_begin, st.n_languages, st.transcribe, st.translate,
                  st.notimestamps, gen.suppress_tokens, gen.begin_suppress_tokens, multilingual=False)
    clips = _clips()
    for i, name in enumerate(("speech30", "noise12")):
        toks, _ = wo.generate(tiny_oracle, wo.log_mel(clips[name], TINY.n_mels), g, task=None, return_timestamps=True,
                              max_new_tokens=48)
        ref = [int(t) for t in tiny_golden["gen_sequences"][i]]
        while ref and ref[-1] == st.eot:
            ref.pop()
        assert toks == ref, (name, toks, ref)


def test_fallback_criteria_match_transformers(oracle_model, gcfg):
    """oracle.pass_criteria (compression ratio, avg logprob of the processed scores, no-speech probability) against
    the values transformers' own _need_fallback saw on the first seek pass of every window (tests/golden/
    fallback.json, make_golden.py fallback)."""
    import json

    z = json.load(open(os.path.join(G, "fallback.json")))
    clips = _clips()
    calls = z["metrics"]["calls"][:3]  # the first pass: all three windows, seek 0, batch index = window
    for i, name in enumerate(z["clips"]):
        c = calls[i]
        assert c["index"] == i
        feats = wo.log_mel(clips[name], 128)
        lang = wo.detect_language(oracle_model, oracle_model.encode(feats), gcfg)
        cr, lp, nsp = wo.pass_criteria(oracle_model, feats, gcfg, [gcfg.sot, lang, gcfg.transcribe], c["tokens"])
        assert cr == c["compression_ratio"]
        assert abs(lp - c["avg_logprob"]) < 1e-3, (name, lp, c["avg_logprob"])
        assert abs(nsp - c["no_speech_prob"]) < 1e-3 * c["no_speech_prob"] + 1e-9, (name, nsp, c["no_speech_prob"])


def test_turbo_beam_and_word_goldens_consistent():
    """Shape / ordering invariants of the large-v3-turbo beam and token-timestamp fixtures (made by
    make_golden.py turbo_beam / turbo_word from transformers; checked against the engine by tests/test_gpu_turbo.py)."""
    zb = np.load(os.path.join(G, "turbo_beam.npz"))
    for tag in ("ts1", "ts0"):
        sc, seq = zb[f"{tag}_fin_score"], zb[f"{tag}_fin_seq"]
        assert sc.shape == (2, 5) and seq.shape[:2] == (2, 5)
        assert np.all(np.diff(sc, axis=1) <= 0)  # finished hypotheses best first
        assert seq.shape[2] <= int(zb[f"{tag}_max_new_tokens"][0])
    zw = np.load(os.path.join(G, "turbo_word.npz"))
    for i in range(2):
        assert zw[f"seq{i}"].shape == zw[f"ts{i}"].shape
        assert np.all(np.isfinite(zw[f"ts{i}"])) and np.all(zw[f"ts{i}"] >= 0)


def test_turbo_bench_golden_and_host_processing():
    """tests/golden/turbo_bench.npz (all 128 positions of 6 bench windows, transformers fp32): consistent with
    turbo.npz where both hold a window, the stored masks reproduce the oracle's processor chain (itself pinned to
    transformers) for histories of every kind, the fp32 token is the processed argmax of its stored top-16, and
    turbo_parity.check_forced_position accepts the fp32 row itself."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import turbo_parity as tp
    zb, z = tp.load_bench(), tp.load()
    d = PRESETS["large-v3-turbo"]
    gen = GenerationSettings.default(d)
    st = gen.special
    g = wo.GenCfg(d.vocab, st.eot, st.sot, st.lang_begin, st.n_languages, st.transcribe, st.translate,
                  st.notimestamps, list(gen.suppress_tokens) + [st.eot], gen.begin_suppress_tokens)
    assert [int(w) for w in zb["windows"]] == [0, 5, 11, 17, 22, 23]
    for w in (0, 23):
        assert np.array_equal(zb[f"w{w}_tokens"], z[f"bench_w{w}_tokens"])
        assert np.array_equal(zb[f"w{w}_top_val"], z[f"bench_w{w}_top_val"])
    rng = np.random.default_rng(0)
    for w in (int(x) for x in zb["windows"]):
        k = f"w{w}_"
        toks = [int(t) for t in zb[k + "tokens"]]
        off = zb[k + "mask_off"]
        assert len(toks) == 128 and len(off) == 129
        for t in list(range(6)) + list(rng.choice(np.arange(6, 128), 10, replace=False)):
            iv = zb[k + "mask_iv"][off[t]: off[t + 1]]
            raw = rng.standard_normal(d.vocab).astype(np.float32) * 3
            raw[st.timestamp_begin:] -= rng.uniform(0, 6)  # both sides of the timestamp rule
            s, margin = tp.process_row(raw, iv, st.timestamp_begin)
            assert np.array_equal(s, wo.process_logits(raw, toks[:t], g, True)), (w, t)
            assert int(zb[k + "top_idx"][t][0]) == toks[t]
            # the fp32 row's own stored top-16, scattered into a row: accepted at distance 0
            row = np.full(d.vocab, -30.0, np.float32)
            row[zb[k + "raw_idx"][t]] = zb[k + "raw_val"][t]
            r = tp.check_forced_position(zb, w, t, row)
            assert r["d_top"] == 0.0

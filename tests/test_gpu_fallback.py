"""Temperature fallback on the MI355X (WhisperGenerationMixin.generate_with_fallback, generation_whisper.py:970-1116):
tw_logits_sample (greedy identical to tw_logits_select; sampling = TemperatureLogitsWarper + TopKLogitsWarper + a
Gumbel-max draw; the chosen tokens' log-probabilities) and tw_token_prob (WhisperNoSpeechDetection), and the engine's
fallback loop against transformers' own criteria values and outcome (tests/golden/fallback.json, made by
make_golden.py fallback).

Tolerances: greedy tokens and processor state bit-exact; per-step log-probabilities 1e-3 (fp32 logits, fp32 vs the
numpy restatement); the pass's average log-probability 0.03 and the no-speech probability 10 % relative against
transformers fp32 (bf16 engine at test-mini, whose logits are within 0.15); sampled tokens: the empirical frequencies
of 8192 draws within 5 sigma of softmax(x / T) over the top-k set, nothing drawn outside it. Sampled sequences are
a valid sampler's output, not torch.multinomial's random stream: parity for them is unpinned."""
import ctypes
import json
import os

import numpy as np
import pytest
import torch

from oracle import whisper_oracle as wo
from twamd import _lib
from twamd.config import PRESETS, GenerationSettings
from twamd.pipeline import TurboTranscriber
from twamd.segments import FallbackConfig
from twamd.synth_audio import silence, speech_like, white_noise

pytestmark = pytest.mark.gpu
DEV = "cuda"
G = os.path.join(os.path.dirname(__file__), "golden")
D = PRESETS["test-mini"]


def S():
    return torch.cuda.current_stream().cuda_stream


def _gcfg():
    gen = GenerationSettings.default(D)
    st = gen.special
    return gen, wo.GenCfg(D.vocab, st.eot, st.sot, st.lang_begin, st.n_languages, st.transcribe, st.translate,
                          st.notimestamps, gen.suppress_tokens, gen.begin_suppress_tokens)


def _params(gen, max_new=40, use_ts=True, V=None):
    st = gen.special
    p = _lib.TwSelectParams()
    p.V, p.eos, p.pad = V or D.vocab, st.eot, st.eot
    p.ts_begin, p.no_timestamps = st.timestamp_begin, st.notimestamps
    p.max_initial_ts = gen.max_initial_timestamp_index
    p.use_timestamps, p.max_new, p.mode = int(use_ts), max_new, 0
    p.lo, p.hi = st.lang_begin, st.lang_end
    p.n_begin_suppress = len(gen.begin_suppress_tokens)
    for i, t in enumerate(gen.begin_suppress_tokens):
        p.begin_suppress[i] = t
    return p


def _suppress_bits(tokens, V):
    bits = np.zeros((V + 31) // 32, np.uint32)
    for t in tokens:
        bits[t >> 5] |= np.uint32(1) << np.uint32(t & 31)
    return torch.from_numpy(bits.view(np.int32)).to(DEV)


def _fresh_state(R):
    st = torch.zeros(R, _lib.TW_STATE_STRIDE, dtype=torch.int32, device=DEV)
    st[:, _lib.TW_ST_LAST:_lib.TW_ST_LASTTS + 1] = -1
    return st


def test_sample_greedy_equals_select_and_logprob():
    """temperature 0: tw_logits_sample picks tw_logits_select's token and evolves the processor state identically, over
    30 steps of random logits whose timestamp block is often dominant (the rule, the pair masks, max_initial);
    state[SUMLP] = the sum of log_softmax(processed)[token] of the numpy processor restatement."""
    gen, g = _gcfg()
    R, V, T = 6, D.vocab, 64
    p = _params(gen, max_new=30)
    sb = _suppress_bits(gen.suppress_tokens, V)
    sa, sb2 = _fresh_state(R), _fresh_state(R)
    toka = torch.zeros(R, T, dtype=torch.int32, device=DEV)
    tokb = torch.zeros_like(toka)
    ida, idb = torch.zeros(R, dtype=torch.int32, device=DEV), torch.zeros(R, dtype=torch.int32, device=DEV)
    ws = torch.empty(R, _lib.TW_SELECT_WS_PER_ROW, device=DEV)
    rng = np.random.default_rng(5)
    ref_lp = np.zeros(R)
    hist = [[] for _ in range(R)]
    done = [False] * R
    for step in range(30):
        x = rng.standard_normal((R, V)).astype(np.float32) * 2
        x[:, g.ts_begin:] += rng.choice([-4.0, 0.5, 3.0], size=(R, 1)).astype(np.float32)
        lg = torch.from_numpy(x).to(DEV)
        _lib.call("tw_logits_select", lg.data_ptr(), R, V, sb.data_ptr(), ctypes.byref(p), sa.data_ptr(),
                  toka.data_ptr(), T, ida.data_ptr(), None, ws.data_ptr(), S())
        _lib.call("tw_logits_sample", lg.data_ptr(), R, V, sb.data_ptr(), ctypes.byref(p), 0.0, 50, 7, None,
                  sb2.data_ptr(), tokb.data_ptr(), T, idb.data_ptr(), None, S())
        torch.cuda.synchronize()
        assert torch.equal(toka[:, step], tokb[:, step]), step
        assert torch.equal(sa[:, :6], sb2[:, :6]), step
        for r in range(R):
            tok = int(tokb[r, step])
            if not done[r]:
                s = wo.process_logits(x[r], hist[r], g, True)
                fin = s[np.isfinite(s)]
                m = fin.max()
                ref_lp[r] += s[tok] - (m + np.log(np.exp(fin - m).sum()))
                hist[r].append(tok)
                done[r] = tok == g.eot or len(hist[r]) >= 30
    got = sb2[:, _lib.TW_ST_SUMLP].cpu().view(torch.float32).numpy()
    np.testing.assert_allclose(got, ref_lp, atol=1e-3 * 30, rtol=0)


def test_sampler_distribution_topk_and_temperature():
    """8192 rows of the same logits (no timestamps, V = 2048), one draw each (the row key varies): the frequencies
    follow softmax(x / T) over the 50 largest (the k-th value's ties kept), nothing outside; SUMLP = x[tok] - the
    kept set's logsumexp (scores * T, _retrieve_avg_logprobs)."""
    gen, _ = _gcfg()
    V, R, T, K = 2048, 8192, 0.7, 50
    rng = np.random.default_rng(11)
    x = rng.standard_normal(V).astype(np.float32) * 1.5
    x[rng.choice(V, 80, replace=False)] += 4.0
    x[7] = x[9]  # a tie somewhere
    p = _params(gen, max_new=4, use_ts=False, V=V)
    p.n_begin_suppress = 0
    lg = torch.from_numpy(np.tile(x, (R, 1))).to(DEV)
    st = _fresh_state(R)
    st[:, _lib.TW_ST_NGEN] = 1  # (not the first step: no begin-suppression)
    tok = torch.zeros(R, 8, dtype=torch.int32, device=DEV)
    ids = torch.zeros(R, dtype=torch.int32, device=DEV)
    keys = torch.arange(R, dtype=torch.int32, device=DEV)
    _lib.call("tw_logits_sample", lg.data_ptr(), R, V, None, ctypes.byref(p), T, K, 12345, keys.data_ptr(),
              st.data_ptr(), tok.data_ptr(), 8, ids.data_ptr(), None, S())
    torch.cuda.synchronize()
    draws = ids.cpu().numpy()
    kth = np.sort(x)[::-1][K - 1]
    keep = x >= kth
    assert keep[draws].all(), "a token outside the top-k set was drawn"
    pr = np.where(keep, np.exp((x - x.max()) / T), 0.0)
    pr /= pr.sum()
    freq = np.bincount(draws, minlength=V) / R
    sig = np.sqrt(pr * (1 - pr) / R)
    assert np.all(np.abs(freq - pr) <= 5 * sig + 1e-4), np.abs(freq - pr).max()
    kx = x[keep].astype(np.float64)
    lse = kx.max() + np.log(np.exp(kx - kx.max()).sum())
    lp = st[:, _lib.TW_ST_SUMLP].cpu().view(torch.float32).numpy()
    np.testing.assert_allclose(lp, x[draws] - lse, atol=1e-4)
    # the same key and seed draw the same token; another seed draws differently somewhere
    st2 = _fresh_state(R)
    st2[:, _lib.TW_ST_NGEN] = 1
    ids2 = torch.zeros_like(ids)
    _lib.call("tw_logits_sample", lg.data_ptr(), R, V, None, ctypes.byref(p), T, K, 12345, keys.data_ptr(),
              st2.data_ptr(), tok.data_ptr(), 8, ids2.data_ptr(), None, S())
    ids3 = torch.zeros_like(ids)
    st3 = _fresh_state(R)
    st3[:, _lib.TW_ST_NGEN] = 1
    _lib.call("tw_logits_sample", lg.data_ptr(), R, V, None, ctypes.byref(p), T, K, 999, keys.data_ptr(),
              st3.data_ptr(), tok.data_ptr(), 8, ids3.data_ptr(), None, S())
    torch.cuda.synchronize()
    assert torch.equal(ids, ids2) and not torch.equal(ids, ids3)


def test_token_prob_kernel():
    R, V = 5, D.vocab
    x = torch.randn(R, V, device=DEV) * 3
    st = _fresh_state(R)
    _lib.call("tw_token_prob", x.data_ptr(), R, V, V, 50361, st.data_ptr(), S())
    got = st[:, _lib.TW_ST_NOSPEECH].cpu().view(torch.float32)
    ref = torch.softmax(x.double(), -1)[:, 50361].cpu().float()
    torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-9)


# ---- the engine's fallback loop vs transformers ----------------------------------------------------------------------
@pytest.fixture(scope="module")
def mini():
    return TurboTranscriber.from_pretrained("test-mini", seed=1234, max_batch=4)


@pytest.fixture(scope="module")
def fz():
    return json.load(open(os.path.join(G, "fallback.json")))


def _load3(tr):
    eng = tr.engine
    clips = [speech_like(30.0, 1234), white_noise(12.3, 7), silence(30.0)]
    host = np.zeros((3, 480000), np.float32)
    for i, c in enumerate(clips):
        host[i, : len(c)] = c[:480000]
    eng.wave[:3].copy_(torch.from_numpy(host))
    eng.logmel(3)


def test_first_pass_criteria_vs_transformers(mini, fz):
    """sample_pass at temperature 0 over the three windows: the greedy tokens, their average log-probability and the
    no-speech probability against the values transformers' _need_fallback saw on the first seek pass."""
    eng = mini.engine
    _load3(mini)
    eng.row_map[:3] = torch.arange(3, dtype=torch.int32)
    eng.seek[:3] = 0
    eng.encode(3)
    st = mini.gen.special
    tail = eng.prompt_tail("transcribe", True)
    res = eng.sample_pass(3, tail, None, 40, temperature=0.0, no_speech_token=st.notimestamps - 1)
    for i, c in enumerate(fz["metrics"]["calls"][:3]):
        toks = [int(t) for t in res.tokens[i]]
        n = toks.index(st.eot) + 1 if st.eot in toks else len(toks)
        ref = c["tokens"]
        avg = res.sum_logprob[i] / n
        print(f"window {i}: tokens equal {toks[:n] == ref}, avg logprob {avg:.4f} vs {c['avg_logprob']:.4f}, "
              f"no-speech {res.no_speech_prob[i]:.3e} vs {c['no_speech_prob']:.3e}")
        if toks[:n] == ref:
            assert abs(avg - c["avg_logprob"]) < 0.03
        assert abs(res.no_speech_prob[i] - c["no_speech_prob"]) <= 0.1 * c["no_speech_prob"]


def test_no_speech_skip_matches_transformers(mini, fz):
    """FALLBACK_SKIP (temperature (0.0,), logprob_threshold -3, no_speech_threshold 3e-5): the silent window's first
    pass is skipped, the other two keep their greedy tokens: generate()'s sequences exactly."""
    eng = mini.engine
    _load3(mini)
    kw = fz["skip"]["kwargs"]
    fb = FallbackConfig(temperatures=tuple(kw["temperature"]), logprob_threshold=kw["logprob_threshold"],
                        no_speech_threshold=kw["no_speech_threshold"])
    seqs = eng.generate(3, task="transcribe", max_new_tokens=40, return_timestamps=True, fallback=fb)
    eot = mini.gen.special.eot
    for i, ref in enumerate(fz["skip"]["sequences"]):
        ref = [t for t in ref]
        while ref and ref[-1] == eot:
            ref.pop()
        assert seqs[i] == ref, (i, seqs[i][:8], ref[:8])
    assert seqs[2] == []


def test_temperature_fallback_resamples_failing_windows(mini):
    """temperature (0.0, 0.7) with logprob_threshold -3: windows 0 and 2 (first-pass average log-probabilities -3.37
    and -3.19 in fp32) are re-decoded by sampling, window 1 (-2.64) keeps its greedy tokens; the draw is a function of
    the seed; the pipeline accepts the transformers kwargs and rejects unknown ones."""
    eng = mini.engine
    _load3(mini)
    greedy = eng.generate(3, task="transcribe", max_new_tokens=40, return_timestamps=True, max_passes=1)
    out = {}
    for seed in (1, 1, 2):
        _load3(mini)
        fb = FallbackConfig(temperatures=(0.0, 0.7), logprob_threshold=-3.0, seed=seed)
        out.setdefault(seed, []).append(eng.generate(3, task="transcribe", max_new_tokens=40, return_timestamps=True,
                                                     fallback=fb, max_passes=1))
    a, b = out[1]
    assert a == b
    assert a[1] == greedy[1]
    assert a[0] != greedy[0] or a[2] != greedy[2]
    assert out[2][0] != a
    tsb = mini.gen.special.timestamp_begin
    for s in a:  # the timestamp processor still holds: timestamps come in non-decreasing order
        ts = [t for t in s if t >= tsb]
        assert ts == sorted(ts)
    audio = speech_like(30.0, 1234)
    r = mini(audio, chunk_length_s=30, stride_length_s=0, return_timestamps=True,
             generate_kwargs={"num_beams": 1, "temperature": (0.0, 0.7), "logprob_threshold": -3.0,
                              "max_new_tokens": 40})
    assert "text" in r and "chunks" in r
    with pytest.raises(ValueError, match="not supported"):
        mini(audio, chunk_length_s=30, generate_kwargs={"num_beams": 1, "bogus_kwarg": 1})
    r = mini(audio, chunk_length_s=30, generate_kwargs={"temperature": (0.0, 0.2), "logprob_threshold": -1.0,
                                                         "max_new_tokens": 24})  # (the default decode: beam-5)
    assert "text" in r


# ---- the fallback with beam search (num_beams = 3) vs transformers (tests/golden/fallback_beam.json) ----------------
@pytest.fixture(scope="module")
def fbz():
    return json.load(open(os.path.join(G, "fallback_beam.json")))


def test_beam_first_pass_criteria_vs_transformers(mini, fbz):
    """beam_pass(criteria=True) over the three windows: the best hypotheses, their average log-probability from the
    scores renormalised over the allowed tokens (what _retrieve_avg_logprobs takes from the processed beam scores) and
    the no-speech probability at <|startoftranscript|>, against the values transformers' _need_fallback saw on the
    first seek pass with num_beams=3."""
    eng = mini.engine
    _load3(mini)
    eng.row_map[:3] = torch.arange(3, dtype=torch.int32)
    eng.seek[:3] = 0
    eng.encode(3)
    st = mini.gen.special
    tail = eng.prompt_tail("transcribe", True)
    res = eng.beam_pass(3, 3, tail, None, 24, criteria=True, no_speech_token=st.notimestamps - 1)
    compared = 0
    for i, c in enumerate(fbz["metrics"]["calls"][:3]):
        toks = [int(t) for t in res.tokens[i]]
        ref = c["tokens"]
        avg = res.sum_logprob[i] / len(toks)
        print(f"window {i}: tokens equal {toks == ref}, avg logprob {avg:.4f} vs {c['avg_logprob']:.4f}, "
              f"no-speech {res.no_speech_prob[i]:.3e} vs {c['no_speech_prob']:.3e}")
        if toks == ref:
            assert abs(avg - c["avg_logprob"]) < 0.03
            compared += 1
        assert abs(res.no_speech_prob[i] - c["no_speech_prob"]) <= 0.1 * c["no_speech_prob"]
    assert compared >= 2


def test_beam_fallback_outcome_matches_transformers(mini, fbz):
    """FALLBACK_SKIP with num_beams=3 (one temperature: the criteria are evaluated, nothing re-decodes): generate()'s
    sequences."""
    eng = mini.engine
    _load3(mini)
    kw = fbz["skip"]["kwargs"]
    fb = FallbackConfig(temperatures=tuple(kw["temperature"]), logprob_threshold=kw["logprob_threshold"],
                        no_speech_threshold=kw["no_speech_threshold"])
    seqs = eng.generate(3, task="transcribe", max_new_tokens=24, return_timestamps=True, fallback=fb, num_beams=3)
    eot = mini.gen.special.eot
    for i, ref in enumerate(fbz["skip"]["sequences"]):
        ref = list(ref)
        while ref and ref[-1] == eot:
            ref.pop()
        assert seqs[i] == ref, (i, seqs[i][:8], ref[:8])


def test_beam_fallback_sampling_round_turns_the_call_greedy(mini, fbz):
    """temperature (0.0, 0.4), logprob_threshold -2.5, num_beams=3: the first pass's beam round fails every window
    (as transformers' decisions in fallback_beam.json "resample"), the retry samples, and from then on the call decodes
    without beams (transformers leaves generation_config.num_beams = 1): exactly one beam search in the call."""
    eng = mini.engine
    _load3(mini)
    calls = fbz["resample"]["calls"]
    assert [c["num_beams"] for c in calls][:3] == [3, 3, 3] and all(c["num_beams"] == 1 for c in calls[3:])
    kw = fbz["resample"]["kwargs"]
    fb = FallbackConfig(temperatures=tuple(kw["temperature"]), logprob_threshold=kw["logprob_threshold"], seed=3)
    n_beam = []
    orig = eng.beam_pass

    def counting(*a, **k):
        n_beam.append(a[0])
        return orig(*a, **k)

    eng.beam_pass = counting
    try:
        seqs = eng.generate(3, task="transcribe", max_new_tokens=24, return_timestamps=True, fallback=fb, num_beams=3,
                            max_passes=3)
    finally:
        del eng.beam_pass
    assert n_beam == [3], n_beam
    assert all(isinstance(s, list) for s in seqs)

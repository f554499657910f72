"""Call options combined (tests/golden/word_combos.json, transformers' ASR pipeline at test-mini on 75 s of audio):
word-level timestamps on a long-form input, with condition_on_prev_tokens (chunked batch and long-form), with the
temperature-fallback criteria, and the fallback criteria with beam search.

Pass criterion per case: the pipeline output equals transformers', or — where bf16 arithmetic took the other side of
a near-tie of this random-weight model — every greedy device decision is within TAU logits of the fp32 oracle
replaying the device's passes (with the prompts it fed and the input's frame count), and, for beams, the first
decision where the device leaves the fp32 beam search is one that search could make within tolerance. Word chunk
times, where the transcript is transformers': every one within 0.5 s, and >= 90 % exactly equal or the differing ones
in at most one contiguous run per 20 times (a DTW jump moves the run of boundaries it crosses: on MI355X long_cond_word
moves 4 of 18 times, two zero-length words at one boundary, by 0.06 s). (The fp32 oracle's
long-form word times equal transformers' exactly — checked on the CPU, oracle.generate_batch_word with max_frames —
and the device's differ at one zero-length word by 0.46 s: one DTW jump across flat attention, where the bf16
attention of the alignment heads ranks two near-equal paths the other way.)"""
import json
import os

import numpy as np
import pytest

from oracle import whisper_oracle as wo
from twamd.config import PRESETS, GenerationSettings
from twamd.pipeline import TurboTranscriber
from twamd.synth_audio import speech_like, white_noise

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")
D = PRESETS["test-mini"]
TAU = 0.3


@pytest.fixture(scope="module")
def gold():
    with open(os.path.join(G, "word_combos.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def tr(gold):
    t = TurboTranscriber.from_pretrained("test-mini", seed=1234, max_batch=3)
    t.engine.gen.alignment_heads = [tuple(h) for h in gold["alignment_heads"]]
    return t


@pytest.fixture(scope="module")
def oracle():
    sd = wo.synth_state_dict(D.d_model, D.encoder_layers, D.decoder_layers, D.ffn, D.n_mels, D.vocab, 1234)
    return wo.WhisperOracle(sd, D.heads)


def _gcfg():
    gen = GenerationSettings.default(D)
    st = gen.special
    return wo.GenCfg(D.vocab, st.eot, st.sot, st.lang_begin, st.n_languages, st.transcribe, st.translate,
                     st.notimestamps, gen.suppress_tokens, gen.begin_suppress_tokens)


def _close_times(got, ref, what):
    got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    assert got.shape == ref.shape, what
    if got.size:
        d = np.abs(got - ref)
        print(f"{what}: {d.size} word times, {(d < 1e-6).mean():.0%} equal, max |d| {d.max():.2f} s")
        assert d.max() <= 0.5 + 1e-6, (what, float(d.max()))
        # the differing times come in runs, one per DTW jump (a jump moves every boundary it crosses): >= 90 % of the
        # times exactly equal, or at most one jump per 20 word times
        diff = np.flatnonzero(d >= 1e-6)
        jumps = int(diff.size > 0) + int(np.count_nonzero(np.diff(diff) > 1))
        assert (d < 1e-6).mean() >= 0.9 or jumps <= max(1, d.size // 20), (what, jumps, float((d < 1e-6).mean()))


@pytest.mark.parametrize("name", ["long_word", "cond_word", "fallback_word", "long_cond_word", "fallback_beam3"])
def test_combined_call_options_match_transformers(tr, oracle, gold, name):
    from twamd.frontend import chunk_windows

    case = next(c for c in gold["cases"] if c["name"] == name)
    x = np.concatenate([speech_like(40.0, 5), white_noise(35.0, 11)]).astype(np.float32)
    gk = dict(case["generate_kwargs"])
    r = tr(x.copy(), generate_kwargs=dict(gk), return_timestamps=case["return_timestamps"], **case["kwargs"])
    exp = case["output"]
    got = json.loads(json.dumps(r))
    if got == exp:
        print(f"{name}: exact")
        return
    word = case["return_timestamps"] == "word"
    if word and r["text"] == exp["text"]:
        assert [c["text"] for c in r["chunks"]] == [c["text"] for c in exp["chunks"]], name
        _close_times([t for c in r["chunks"] for t in c["timestamp"]],
                     [t for c in exp["chunks"] for t in c["timestamp"]], name)
        print(f"{name}: same transcript, word times within the bound")
        return
    print(f"{name}: differs from transformers' (near-tie): {r['text'][:70]!r}")
    if gk.get("num_beams", 1) > 1:
        import test_gpu_e2e as e2e
        e2e._beam_passes_within_tau(tr, oracle, x, case["kwargs"], gk["task"], gk["max_new_tokens"],
                                    num_beams=gk["num_beams"])
        return
    g = _gcfg()
    kw = case["kwargs"]
    if kw.get("chunk_length_s"):
        wins = list(chunk_windows(len(x), kw["chunk_length_s"], kw.get("stride_length_s"), 16000))
        feats = [(wo.log_mel(x[w.start: w.start + min(w.length, 480000)], D.n_mels), 3000) for w in wins]
    else:
        f = wo.log_mel(x, D.n_mels, long=True)
        feats = [(f, f.shape[1])]
    cond = bool(gk.get("condition_on_prev_tokens"))
    for k, (f, T) in enumerate(feats):
        pf = [None if p is None else (list(p[0]), int(p[1])) for p in tr.last_window_prefixes[k]] if cond else None
        st = wo.replay_generate(oracle, f, g, tr.last_window_passes[k], tr.last_window_langs[k],
                                max_new_tokens=gk["max_new_tokens"], tau=TAU, max_frames=T, prefixes=pf)
        assert st["ok"], (name, k, st)

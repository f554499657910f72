"""Long-form input and condition_on_prev_tokens, host side (CPU), against tests/golden/longform.json (transformers'
ASR pipeline at test-mini on 75 s of audio without chunk_length_s, and with condition_on_prev_tokens=True; every seek
pass's decoder prompt and raw output spied from generate_with_fallback):

  * the oracle's long-form log-mel (one STFT over the whole input, the max - 8 clamp over all of it) equals the
    feature extractor's with truncation=False, padding="longest" (asr:450-457);
  * twamd.segments.condition_prefixes + segment_slices rebuild every conditioned prompt transformers built from the
    previous passes' outputs (generation_whisper.py:1853-1918, _pad_to_max_length's left padding, the double-ending
    timestamp skip, the <|startofprev|> token, the current_segments[0] gate), token for token;
  * the seek bookkeeping of a long input (max_frames = the input's frames, seek_num_frames = min(T - seek, 3000))
    reproduces the passes' seek positions.
"""
import json
import os

import numpy as np
import pytest

from oracle import whisper_oracle as wo
from twamd.config import PRESETS, GenerationSettings
from twamd.segments import condition_prefixes, retrieve_segment, segment_slices
from twamd.synth_audio import speech_like, white_noise

G = os.path.join(os.path.dirname(__file__), "golden")
D = PRESETS["test-mini"]


@pytest.fixture(scope="module")
def gold():
    with open(os.path.join(G, "longform.json")) as f:
        return json.load(f)


def _audio():
    return np.concatenate([speech_like(40.0, 5), white_noise(35.0, 11)]).astype(np.float32)


def test_long_form_log_mel_matches_feature_extractor(gold):
    x = _audio()
    assert len(x) == gold["n_samples"]
    f = wo.log_mel(x, D.n_mels, long=True)
    assert list(f.shape) == gold["features"]["shape"]  # n // 160 frames
    np.testing.assert_allclose(f[:, ::97], np.array(gold["features"]["sub"], np.float32), atol=1e-4)
    np.testing.assert_allclose(f.sum(axis=0)[::7], np.array(gold["features"]["colsum"]), atol=5e-3)


def _prev_sot(gen):
    return gen.prev_sot_token_id if gen.prev_sot_token_id is not None else gen.suppress_tokens[-2]


@pytest.mark.parametrize("name", ["long_cond", "chunk30_cond_b3"])
def test_condition_prompts_rebuilt_from_previous_passes(gold, name):
    gen = GenerationSettings.default(D)
    st = gen.special
    case = next(c for c in gold["cases"] if c["name"] == name)
    passes = case["passes"]
    assert len(passes) >= 3
    n = len(passes[0]["rows"])
    segs = [[] for _ in range(n)]
    checked = 0
    for p in passes:
        rows = p["rows"]
        init = [q[-3:] for q in p["prompts"]]  # SOT, language, task (timestamps on)
        if len(segs[0]) > 0:  # transformers gates on the batch's first row (generation_whisper.py:1883)
            pref, pads = condition_prefixes([segs[i] for i in rows], _prev_sot(gen), st.eot, st.timestamp_begin,
                                            448 // 2 - 1)
            want = [q[:-3] for q in p["prompts"]]
            assert pref == want, (name, p["seek"])
            assert pads == [len(q) - len(q[k:]) for q in pref for k in [next(k for k, t in enumerate(q) if t != st.eot)]]
            checked += 1
        else:
            assert all(len(q) == 3 for q in p["prompts"])
        for j, i in enumerate(rows):
            seq = p["sequences"][j]
            segs[i].extend(segment_slices(seq, st.timestamp_begin))
            toks, _ = retrieve_segment(seq, 0, 3000, st.timestamp_begin)
            assert sum(segment_slices(seq, st.timestamp_begin), []) == toks
        assert all(len(q) == 3 for q in init)
    assert checked >= 2


def test_condition_prefix_pads_and_cut_off():
    tb = 100
    body = [1 + k % 90 for k in range(299)]
    segs = [[[101, 5, 6, 102, 103]], None, [], [[100] + body + [120]]]
    rows, pads = condition_prefixes(segs, 99, 0, tb, 223)
    L = max(len(r) for r in rows)
    assert all(len(r) == L for r in rows) and L == 224  # <|startofprev|> + the last 223 tokens
    assert rows[0][-5:] == [99, 101, 5, 6, 102]  # a segment ending in two timestamps loses the last one
    assert rows[1][-1:] == [99] and rows[2][-1:] == [99]  # unconditioned / no segments: <|startofprev|> alone
    assert pads == [L - 5, L - 1, L - 1, 0]
    assert rows[3][1:] == (body + [120])[-223:]
    rows2, pads2 = condition_prefixes([None, []], None, 0, tb, 223)
    assert rows2 == [[], []] and pads2 == [0, 0]


def test_long_form_seek_positions(gold):
    """The spied passes' seek positions follow retrieve_segment with seek_num_frames = min(T - seek, 3000)."""
    gen = GenerationSettings.default(D)
    st = gen.special
    T = gold["features"]["shape"][1]
    for case in gold["cases"]:
        if case["kwargs"]:
            continue
        seek = 0
        for p in case["passes"]:
            assert p["seek"] == [seek], case["name"]
            _, off = retrieve_segment(p["sequences"][0], seek, min(T - seek, 3000), st.timestamp_begin)
            seek += off
        assert seek >= T


def test_oracle_long_form_word_timestamps_match_transformers():
    """The oracle's generate_batch_word over a long-form input (max_frames = the input's frames, num_frames = the
    feature extractor's attention mask length ceil(n / 160)) through the host's decode_asr equals the transformers
    pipeline's return_timestamps="word" output on 75 s without chunking (word_combos.json "long_word") exactly: the
    semantics the engine's long-form word path follows."""
    from twamd.frontend import time_precision
    from twamd.tokenizer import WhisperVocab, decode_asr

    gold = json.load(open(os.path.join(G, "word_combos.json")))
    case = next(c for c in gold["cases"] if c["name"] == "long_word")
    gen = GenerationSettings.default(D)
    st = gen.special
    g = wo.GenCfg(D.vocab, st.eot, st.sot, st.lang_begin, st.n_languages, st.transcribe, st.translate,
                  st.notimestamps, gen.suppress_tokens, gen.begin_suppress_tokens)
    m = wo.WhisperOracle(wo.synth_state_dict(D.d_model, D.encoder_layers, D.decoder_layers, D.ffn, D.n_mels, D.vocab,
                                             1234), D.heads)
    x = _audio()
    f = wo.log_mel(x, D.n_mels, long=True)
    heads = [tuple(h) for h in gold["alignment_heads"]]
    (toks, _, tts), = wo.generate_batch_word(m, [f], g, heads, [-(-len(x) // 160)], max_new_tokens=40,
                                             max_frames=[f.shape[1]])
    text, opt = decode_asr(WhisperVocab.synthetic(st), [{"tokens": toks, "token_timestamps": tts}],
                           return_timestamps="word", return_language=False, time_precision=time_precision(1500))
    assert json.loads(json.dumps({"text": text, **opt})) == case["output"]

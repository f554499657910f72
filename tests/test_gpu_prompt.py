"""prompt_ids through the engine (tests/golden/prompt.json, transformers' ASR pipeline at test-mini on 75 s of audio):
chunked 30-s windows in a batch of 3 and long-form, unconditioned and with condition_on_prev_tokens under both
prompt_condition_type values, with and without timestamps.

Pass criterion per case: the pipeline output equals transformers', or — where bf16 arithmetic took the other side of a
near-tie of this random-weight model — every greedy device decision is within TAU logits of the fp32 oracle replaying
the device's passes with the prompts it fed (tests/test_gpu_longform.py's rule). Also: the prompt the device fed each
pass equals the one transformers fed it wherever the device's previous passes equal transformers', the language is
detected without the prompt, and the option checks of _set_prompt_condition_type (generation_whisper.py:1732-1748)."""
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
    with open(os.path.join(G, "prompt.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def tr(gold):
    t = TurboTranscriber.from_pretrained("test-mini", seed=1234, max_batch=3)
    t.engine.gen.prev_sot_token_id = gold["prompt_ids"][0]  # (the golden's generation_config.prev_sot_token_id)
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


def _audio():
    return np.concatenate([speech_like(40.0, 5), white_noise(35.0, 11)]).astype(np.float32)


@pytest.mark.parametrize("name", ["chunk30_prompt_b3", "long_prompt", "long_prompt_cond", "long_prompt_all",
                                  "chunk30_prompt_no_ts"])
def test_prompt_ids_match_transformers(tr, oracle, gold, name):
    from twamd.frontend import chunk_windows

    case = next(c for c in gold["cases"] if c["name"] == name)
    x = _audio()
    gk = dict(case["generate_kwargs"], prompt_ids=np.array(gold["prompt_ids"]))
    r = tr(x.copy(), generate_kwargs=gk, return_timestamps=case["return_timestamps"], **case["kwargs"])
    exp = case["output"]
    # the first pass's prompt of every window is transformers' (no earlier pass to differ from)
    first = case["passes"][0]
    ninit = 3 if case["return_timestamps"] else 4
    for j, i in enumerate(first["rows"]):
        fed = tr.last_window_prefixes[i][0] if len(tr.last_window_prefixes) > i else None
        if fed is not None:
            assert list(fed[0])[fed[1]:] == first["prompts"][j][:-ninit], (name, i)
    got = json.loads(json.dumps(r))
    if got == exp:
        print(f"{name}: exact; passes {[len(p) for p in tr.last_window_passes]}")
        return
    print(f"{name}: differs from transformers' (near-tie): {r['text'][:70]!r}")
    g = _gcfg()
    kw = case["kwargs"]
    if kw.get("chunk_length_s"):
        wins = list(chunk_windows(len(x), kw["chunk_length_s"], kw.get("stride_length_s"), 16000))
        feats = [(wo.log_mel(x[w.start: w.start + min(w.length, 480000)], D.n_mels), 3000) for w in wins]
    else:
        f = wo.log_mel(x, D.n_mels, long=True)
        feats = [(f, f.shape[1])]
    for k, (f, T) in enumerate(feats):
        pf = [None if p is None else (list(p[0]), int(p[1])) for p in tr.last_window_prefixes[k]]
        st = wo.replay_generate(oracle, f, g, tr.last_window_passes[k], tr.last_window_langs[k],
                                return_timestamps=bool(case["return_timestamps"]), max_new_tokens=gk["max_new_tokens"],
                                tau=TAU, max_frames=T, prefixes=pf)
        assert st["ok"], (name, k, st)


def test_prompt_condition_type_checks(tr):
    x = _audio()[:16000 * 20]
    p = np.array([tr.engine.gen.prev_sot_token_id, 1000, 2000])
    with pytest.raises(ValueError, match="condition_on_prev_tokens=True"):
        tr(x, generate_kwargs={"prompt_ids": p, "prompt_condition_type": "all-segments", "max_new_tokens": 8})
    with pytest.raises(ValueError, match="does not exist"):
        tr(x, generate_kwargs={"prompt_ids": p, "prompt_condition_type": "every-segment", "max_new_tokens": 8})

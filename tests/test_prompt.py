"""prompt_ids (generate()'s initial prompt), host side (CPU), against tests/golden/prompt.json (transformers' ASR pipeline
at test-mini on 75 s of audio with prompt_ids = [<|startofprev|>, 1000, ..., 6000]; every seek pass's decoder prompt and
raw output spied from generate_with_fallback, tests/golden/make_golden.py make_prompt):

  * the engine's rule for a pass's prompt prefix — unconditioned: prompt_ids in front of every pass
    (generation_whisper.py:1909-1912); conditioned, "first-segment": the prompt (without <|startofprev|>) is every
    chunk's first segment (_prepare_segments, :1119-1124) and goes through condition_prefixes with the rest;
    "all-segments": the first pass takes prompt_ids, later ones prompt_ids + the previous segments (:1887-1888) —
    rebuilds every prompt transformers built, token for token.
The engine side (outputs, the option checks of _set_prompt_condition_type) is tests/test_gpu_prompt.py.
"""
import json
import os

import pytest

from twamd.config import PRESETS, GenerationSettings
from twamd.segments import condition_prefixes, segment_slices

G = os.path.join(os.path.dirname(__file__), "golden")
D = PRESETS["test-mini"]


@pytest.fixture(scope="module")
def gold():
    with open(os.path.join(G, "prompt.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("name", ["chunk30_prompt_b3", "long_prompt", "long_prompt_cond", "long_prompt_all",
                                  "chunk30_prompt_no_ts"])
def test_pass_prompts_rebuilt(gold, name):
    st = GenerationSettings.default(D).special
    case = next(c for c in gold["cases"] if c["name"] == name)
    assert "output" in case, case.get("error")
    gk = case["generate_kwargs"]
    cond = bool(gk.get("condition_on_prev_tokens"))
    all_seg = gk.get("prompt_condition_type") == "all-segments"
    prompt = gold["prompt_ids"]
    prev_sot = prompt[0]  # (the golden's generation_config.prev_sot_token_id)
    passes = case["passes"]
    n = len(passes[0]["rows"])
    seg_lists = [[] for _ in range(n)] if all_seg else [[prompt[1:]] for _ in range(n)]
    ninit = 3 if case["return_timestamps"] else 4  # SOT, language, task (+ notimestamps)
    conditioned = 0
    for p in passes:
        rows = p["rows"]
        want = [q[:-ninit] for q in p["prompts"]]
        if cond and len(seg_lists[0]) > 0:
            pref, _ = condition_prefixes([seg_lists[i] for i in rows], prompt if all_seg else prev_sot, st.eot,
                                         st.timestamp_begin, 448 // 2 - 1)
            conditioned += 1
        else:
            pref = [list(prompt) for _ in rows]
        assert pref == want, (name, p["seek"])
        for j, i in enumerate(rows):
            seg_lists[i].extend(segment_slices(p["sequences"][j], st.timestamp_begin))
    assert conditioned >= (2 if cond else 0)


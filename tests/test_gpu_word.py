"""Word-level timestamps on the GPU path: the alignment-head probabilities written by the
decoder cross-attention kernel (tw_attn_decode_cross_probs), the engine's token-level timestamps against the
batched oracle (oracle/whisper_oracle.py generate_batch_word), and return_timestamps="word" through
TurboTranscriber against the transformers ASR pipeline output (tests/golden/word.json).

Tolerances: the probabilities are f32 softmax over bf16 q.K (|diff| <= 2e-3 relative to the row max). Token
sequences must be identical. The token times come from an argmin path (DTW) over standardized, median-filtered
attention, so bf16 rounding can move a jump by a frame or more where two alignment costs nearly tie: per token
|diff| <= 0.2 s and >= 90 % of the tokens exactly equal (these inputs: see the assertions); word chunks carry the
same text and their times obey the same bound."""
import json
import os

import numpy as np
import pytest
import torch

from oracle import whisper_oracle as wo
from twamd import _lib
from twamd.config import PRESETS, GenerationSettings
from twamd.pipeline import TurboTranscriber
from twamd.synth_audio import speech_like, white_noise

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")
D = PRESETS["test-mini"]
DEV = "cuda"
HEADS = [(1, 0), (1, 1), (1, 2), (1, 3)]


def S():
    return torch.cuda.current_stream().cuda_stream


def test_cross_probs_kernel_vs_torch():
    B, H, Sx, Bt = 3, 6, 1500, 3
    D_ = H * 64
    g = torch.Generator(device="cpu").manual_seed(5)
    ckv = (torch.randn(2, Bt, H, Sx, 64, generator=g) * 0.5).to(torch.bfloat16).to(DEV)
    q = (torch.randn(B, D_, generator=g) * 0.5).to(torch.bfloat16).to(DEV)
    rm = torch.tensor([2, 0, 1], dtype=torch.int32, device=DEV)
    pos = torch.tensor([5, 7, 20], dtype=torch.int32, device=DEV)
    mask, slot0, n_slots, pos0, n_steps = 0b100101, 1, 4, 5, 3  # heads 0, 2, 5 -> slots 1, 2, 3
    probs = torch.full((B, n_steps, n_slots, Sx), float("nan"), dtype=torch.float32, device=DEV)
    out = torch.empty(B, D_, dtype=torch.bfloat16, device=DEV)
    out2 = torch.empty_like(out)
    _lib.call("tw_attn_decode_cross_probs", q.data_ptr(), B, H, Sx, Bt, rm.data_ptr(), ckv.data_ptr(),
              out.data_ptr(), probs.data_ptr(), mask, slot0, n_slots, pos.data_ptr(), pos0, n_steps, S())
    _lib.call("tw_attn_decode_cross", q.data_ptr(), B, H, Sx, Bt, rm.data_ptr(), ckv.data_ptr(), out2.data_ptr(),
              S())
    torch.cuda.synchronize()
    assert torch.equal(out, out2)  # recording the probabilities does not change the attention output
    written = {(0, 0), (1, 2)}  # row 2's step 15 is outside n_steps: nothing written
    for b in range(B):
        s = int(rm[b])
        p = torch.softmax(q[b].float().view(H, 1, 64) @ ckv[0, s].float().transpose(-1, -2), -1)[:, 0]
        for k in range(n_steps):
            for sl in range(n_slots):
                got = probs[b, k, sl]
                if (b, k) in written and sl >= slot0:
                    h = [0, 2, 5][sl - slot0]
                    torch.testing.assert_close(got, p[h], atol=2e-3 * float(p[h].max()), rtol=0)
                else:
                    assert torch.isnan(got).all(), (b, k, sl)


@pytest.fixture(scope="module")
def tr():
    t = TurboTranscriber.from_pretrained("test-mini", seed=1234, max_batch=3)
    t.engine.gen.alignment_heads = list(HEADS)
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
    if got.size == 0:
        return
    d = np.abs(got - ref)
    assert d.max() <= 0.2 + 1e-6, (what, float(d.max()))
    assert (d < 1e-6).mean() >= 0.9, (what, float((d < 1e-6).mean()))


def test_engine_token_timestamps_vs_batched_oracle(tr, oracle):
    # inputs whose greedy tokens have no bf16-vs-fp32 near-ties (token equality is the precondition here)
    clips = [speech_like(30.0, 1234), white_noise(12.3, 7), speech_like(40.0, 5)[: 20 * 16000]]
    eng = tr.engine
    host = np.zeros((len(clips), 480000), np.float32)
    nf = []
    for i, c in enumerate(clips):
        host[i, : len(c)] = c
        nf.append(-(-len(c) // 160))
    eng.wave[: len(clips)].copy_(torch.from_numpy(host))
    eng.logmel(len(clips))
    segs = eng.generate(len(clips), task="transcribe", max_new_tokens=40, word_timestamps=True, num_frames=nf)
    tts = eng.last_token_timestamps
    feats = [wo.log_mel(c, D.n_mels) for c in clips]
    ref = wo.generate_batch_word(oracle, feats, _gcfg(), HEADS, nf, task="transcribe", max_new_tokens=40)
    for i, (toks, _, rts) in enumerate(ref):
        assert segs[i] == toks, i
        _close_times(tts[i], rts, f"window {i}")


def test_pipeline_word_timestamps_match_transformers(tr, oracle):
    """return_timestamps="word" end to end. Where the transcript equals the transformers pipeline's
    (tests/golden/word.json) the word chunks' times are compared with it; where bf16 took the other side of a
    greedy near-tie of this random-weight model (every device decision verified within TAU logits by
    replay_generate, as tests/test_gpu_e2e.py does) the device's per-token times are compared with the oracle's
    times for the device's own tokens (teacher-forced, same batching)."""
    from twamd.frontend import chunk_windows

    TAU = 0.3
    gold = json.load(open(os.path.join(G, "word.json")))
    x = np.concatenate([speech_like(40.0, 5), white_noise(35.0, 11)])
    g = _gcfg()
    for case in gold["cases"]:
        xx = x[: case["n_samples"]]
        kw = dict(case["kwargs"])
        r = tr(xx, generate_kwargs={"task": "transcribe", "num_beams": 1, "max_new_tokens": 40},
               return_timestamps="word", **kw)
        exp = case["output"]
        if r["text"] == exp["text"]:
            assert [c["text"] for c in r["chunks"]] == [c["text"] for c in exp["chunks"]], case["name"]
            got = [t for c in r["chunks"] for t in c["timestamp"]]
            want = [t for c in exp["chunks"] for t in c["timestamp"]]
            _close_times(got, want, case["name"])
            continue
        cl = kw.get("chunk_length_s", 0)
        wins = list(chunk_windows(len(xx), cl, kw.get("stride_length_s"), 16000)) if cl else None
        segs = [xx[w.start: w.start + min(w.length, 480000)] for w in wins] if wins else [xx[:480000]]
        feats = [wo.log_mel(sg, D.n_mels) for sg in segs]
        for k in range(len(segs)):
            st = wo.replay_generate(oracle, feats[k], g, tr.last_window_passes[k], tr.last_window_langs[k],
                                    max_new_tokens=40, tau=TAU)
            assert st["ok"], (case["name"], k, st)
        B = tr.engine.max_batch
        for b0 in range(0, len(segs), B):
            idx = range(b0, min(b0 + B, len(segs)))
            nf = [-(-len(segs[k]) // 160) for k in idx]
            forced = [(tr.last_window_langs[k], tr.last_window_passes[k]) for k in idx]
            ref = wo.generate_batch_word(oracle, [feats[k] for k in idx], g, HEADS, nf, max_new_tokens=40,
                                         forced=forced)
            for k, (toks, _, rts) in zip(idx, ref):
                _close_times(tr.last_window_token_timestamps[k], rts, (case["name"], k))


def _pass_offsets(eng, k=0):
    """Each kept token's seek offset (s) of chunk k's last generate(): the engine's token times carry it (what the
    pipeline consumes), generate()'s top-level token_timestamps do not."""
    from twamd.segments import retrieve_segment, strip_generated

    st = eng.gen.special
    offs, seek = [], 0
    for raw in eng.last_passes[k]:
        seg, adv = retrieve_segment(strip_generated(raw, st.eot), seek, 3000 - seek, st.timestamp_begin)
        offs += [seek * 0.01] * len(seg)
        seek += adv
    return np.asarray(offs)


def test_engine_beam_token_timestamps_vs_transformers(tr):
    """Token-level timestamps of beam search (num_beams=3): the alignment-head cross-attention of the rows that fed
    the best hypothesis (the beam step's finished-hypothesis tables = generate()'s beam_indices), against
    generate(num_beams=3, return_token_timestamps=True) (tests/golden/beam_word.json). Compared where the device's
    beam search returns transformers' tokens; same tolerance as the greedy times."""
    gold = json.load(open(os.path.join(G, "beam_word.json")))
    eng = tr.engine
    eot = eng.gen.special.eot
    clips = {"speech30": speech_like(30.0, 1234), "noise12": white_noise(12.3, 7)}
    compared = 0
    for g in gold["generate"]:
        x = clips[g["clip"]]
        host = np.zeros((1, 480000), np.float32)
        host[0, : len(x)] = x
        eng.wave[:1].copy_(torch.from_numpy(host))
        eng.logmel(1)
        nf = -(-len(x) // 160)
        segs = eng.generate(1, task="transcribe", max_new_tokens=24, num_beams=3, word_timestamps=True,
                            num_frames=[nf])
        ref_t = [int(t) for t in g["sequences"][0]]
        n = len(ref_t)
        while ref_t and ref_t[-1] == eot:
            ref_t.pop()
        if segs[0][: len(ref_t)] != ref_t or len(segs[0]) > n:
            print(f"beam token timestamps {g['clip']}: tokens differ from transformers' (near-tie), not compared")
            continue
        got = (np.asarray(eng.last_token_timestamps[0], np.float64) - _pass_offsets(eng))[: len(ref_t)]
        ref = np.asarray(g["token_timestamps"][0], np.float64)[: len(ref_t)]
        d = np.abs(got - ref)
        print(f"beam token timestamps {g['clip']}: {len(ref_t)} tokens, max |d| {d.max():.3f} s, "
              f"{(d < 1e-4).mean():.0%} equal")
        assert d.max() <= 0.2 + 1e-4 and (d < 1e-4).mean() >= 0.9, (g["clip"], d)
        compared += 1
    assert compared >= 1


def test_pipeline_beam_word_timestamps_match_transformers(tr):
    """return_timestamps="word" with num_beams=3 through the callable against the transformers pipeline (beam_word.json):
    where the transcript is transformers', the word chunks carry the same text and times within the greedy bound."""
    gold = json.load(open(os.path.join(G, "beam_word.json")))
    x = np.concatenate([speech_like(40.0, 5), white_noise(35.0, 11)])
    same = 0
    for case in gold["cases"]:
        xx = x[: case["n_samples"]]
        r = tr(xx, generate_kwargs={"task": "transcribe", "num_beams": 3, "max_new_tokens": 24},
               return_timestamps="word", **case["kwargs"])
        exp = case["output"]
        if r["text"] != exp["text"]:
            print(f"{case['name']}: transcript differs from transformers' (beam near-tie): {r['text'][:60]!r}")
            continue
        assert [c["text"] for c in r["chunks"]] == [c["text"] for c in exp["chunks"]], case["name"]
        _close_times([t for c in r["chunks"] for t in c["timestamp"]],
                     [t for c in exp["chunks"] for t in c["timestamp"]], case["name"])
        same += 1
    assert same >= 1

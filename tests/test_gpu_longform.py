"""Long-form input (> 30 s without chunk_length_s: generate()'s sequential seek loop over the whole input's features)
and condition_on_prev_tokens on the MI355X, through the C-ABI and the product path, against the fp32 oracle and the
transformers pipeline outputs of tests/golden/longform.json (test-mini, seeded weights).

Tolerances: long-form log-mel 1e-4 abs (f32 DFT vs float64 FFT, as the 30-s kernel); encoder rows 0.08 abs (bf16, as
test_gpu_e2e); masked self-attention 2e-2 (bf16 output); transcripts equal to transformers', or every device decision
within 0.3 logits of the fp32 oracle's (replay_generate with the input's frame count and the prompts the device fed).
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import whisper_oracle as wo
from twamd import _lib
from twamd.config import PRESETS, GenerationSettings
from twamd.frontend import dft_basis, mel_table, pack_k8
from twamd.pipeline import TurboTranscriber
from twamd.synth_audio import speech_like, white_noise

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")
D = PRESETS["test-mini"]
DEV = "cuda"
TAU = 0.3


def S():
    return torch.cuda.current_stream().cuda_stream


@pytest.fixture(scope="module")
def tr():
    return TurboTranscriber.from_pretrained("test-mini", seed=1234, max_batch=4)


@pytest.fixture(scope="module")
def oracle():
    sd = wo.synth_state_dict(D.d_model, D.encoder_layers, D.decoder_layers, D.ffn, D.n_mels, D.vocab, 1234)
    return wo.WhisperOracle(sd, D.heads)


@pytest.fixture(scope="module")
def gold():
    with open(os.path.join(G, "longform.json")) as f:
        return json.load(f)


def _gcfg():
    gen = GenerationSettings.default(D)
    st = gen.special
    return wo.GenCfg(D.vocab, st.eot, st.sot, st.lang_begin, st.n_languages, st.transcribe, st.translate,
                     st.notimestamps, gen.suppress_tokens, gen.begin_suppress_tokens)


def _audio():
    return np.concatenate([speech_like(40.0, 5), white_noise(35.0, 11)]).astype(np.float32)


@pytest.mark.parametrize("n", [1200000, 500123, 480001])
def test_logmel_long_vs_oracle(n):
    x = np.concatenate([speech_like(40.0, 5), white_noise(40.0, 3)])[:n].astype(np.float32)
    T = n // 160
    ld = max(T, 3000) + 7
    c, s = dft_basis()
    bc, bs, fb = (torch.from_numpy(pack_k8(a)).to(DEV) for a in (c, s, mel_table(128)))
    feats = torch.full((128, ld), -7.0, device=DEV)
    key = torch.zeros(1, dtype=torch.int32, device=DEV)
    w = torch.from_numpy(x).to(DEV)
    _lib.call("tw_logmel_long", w.data_ptr(), n, bc.data_ptr(), bs.data_ptr(), fb.data_ptr(), 128, feats.data_ptr(), ld,
              key.data_ptr(), S())
    got = feats.cpu().numpy()
    np.testing.assert_allclose(got[:, :T], wo.log_mel(x, 128, long=True), atol=1e-4, rtol=0)
    assert (got[:, T:] == -7.0).all()  # columns past the input's frames untouched


def test_encoder_on_long_input_segments(tr, oracle):
    """Encoder input of a long-form pass = _get_input_segment: feats[:, seek : seek + min(T - seek, 3000)], zero
    padded (tw_im2col_conv1_long), at a seek inside the input and at one whose segment is cut by the input's end."""
    eng = tr.engine
    x = _audio()
    T = eng.set_long_input(torch.from_numpy(x))
    try:
        f = wo.log_mel(x, D.n_mels, long=True)
        for sk in (1234, T - 1700):
            eng.row_map[0] = 0
            eng.seek[0] = sk
            eng.encode(1)
            enc = eng.encoder_output(1)[0].float().cpu().numpy()
            ref = oracle.encode(wo.segment_input(f, sk, T))
            d = np.abs(enc - ref)
            assert d.max() < 0.08 and d.mean() < 0.01, (sk, d.max(), d.mean())
    finally:
        eng.set_long_input(None)


@pytest.mark.parametrize("tab", [False, True])
def test_masked_self_attention_vs_torch(tab):
    """tw_attn_decode_self_masked / _tab_masked: a query at pos >= kv_start attends keys kv_start .. pos; pad queries
    (pos < kv_start) attend 0 .. pos; short (< 256) and long histories (the two-pass form)."""
    torch.manual_seed(5)
    B, H, T = 5, 4, 448
    D_ = H * 64
    pos = torch.tensor([3, 40, 300, 7, 400], dtype=torch.int32, device=DEV)
    ks = torch.tensor([2, 41, 17, 0, 380], dtype=torch.int32, device=DEV)
    kc = torch.randn(B, H, T, 64, device=DEV).to(torch.bfloat16)
    vc = torch.randn(B, H, T, 64, device=DEV).to(torch.bfloat16)
    qkv = (torch.randn(B, 3 * D_, device=DEV) * 0.3).to(torch.bfloat16)
    k0, v0 = kc.clone(), vc.clone()
    out = torch.empty(B, D_, dtype=torch.bfloat16, device=DEV)
    if tab:
        tabt = torch.arange(B, dtype=torch.int32, device=DEV)[:, None].repeat(1, T).contiguous()
        _lib.call("tw_attn_decode_self_tab_masked", qkv.data_ptr(), B, H, T, pos.data_ptr(), kc.data_ptr(),
                  vc.data_ptr(), tabt.data_ptr(), 0, ks.data_ptr(), out.data_ptr(), S())
    else:
        _lib.call("tw_attn_decode_self_masked", qkv.data_ptr(), B, H, T, pos.data_ptr(), kc.data_ptr(), vc.data_ptr(),
                  ks.data_ptr(), out.data_ptr(), S())
    q, k, v = qkv.float().view(B, 3, H, 64).unbind(1)
    for b in range(B):
        t, s0 = int(pos[b]), int(ks[b])
        s0 = s0 if t >= s0 else 0
        K = k0[b].float().clone()
        V = v0[b].float().clone()
        K[:, t] = k[b]
        V[:, t] = v[b]
        sc = torch.einsum("hd,hkd->hk", q[b], K[:, s0: t + 1])
        ref = torch.einsum("hk,hkd->hd", torch.softmax(sc, -1), V[:, s0: t + 1]).reshape(-1)
        torch.testing.assert_close(out[b].float(), ref, atol=2e-2, rtol=2e-2)
        assert torch.equal(kc[b][:, t], k[b].to(torch.bfloat16)) and torch.equal(vc[b][:, t], v[b].to(torch.bfloat16))


def _prefixes_ok(t, k):
    return [None if p is None else (list(p[0]), int(p[1])) for p in t.last_window_prefixes[k]]


@pytest.mark.parametrize("name", ["long_greedy", "long_cond", "long_no_ts", "chunk30_cond_b3"])
def test_long_form_and_conditioning_match_transformers(tr, oracle, gold, name):
    """The pipeline on 75 s without chunking (long-form), with condition_on_prev_tokens, and condition_on_prev_tokens
    over a chunked batch of 3 (left-padded prompts): transformers' output exactly, or every device decision within
    TAU of the fp32 oracle replaying the same passes (and, conditioned, the same prompts)."""
    from twamd.frontend import chunk_windows

    case = next(c for c in gold["cases"] if c["name"] == name)
    x = _audio()
    kw = dict(case["kwargs"])
    if "batch_size" in kw:
        kw["batch_size"] = min(kw["batch_size"], tr.engine.max_batch)
    r = tr(x.copy(), generate_kwargs=dict(case["generate_kwargs"]), return_timestamps=case["return_timestamps"], **kw)
    exact = json.loads(json.dumps(r)) == case["output"]
    print(f"{name}: {'exact' if exact else 'differs'}; passes {[len(p) for p in tr.last_window_passes]}")
    cond = bool(case["generate_kwargs"].get("condition_on_prev_tokens"))
    if cond:  # the device's prompts are the transformers rule applied to its own passes
        assert any(p is not None for w in tr.last_window_prefixes for p in w)
    if exact:
        return
    g = _gcfg()
    if kw.get("chunk_length_s"):
        wins = list(chunk_windows(len(x), kw["chunk_length_s"], kw.get("stride_length_s"), 16000))
        feats = [(wo.log_mel(x[w.start: w.start + min(w.length, 480000)], D.n_mels), 3000) for w in wins]
    else:
        f = wo.log_mel(x, D.n_mels, long=True)
        feats = [(f, f.shape[1])]
    assert len(feats) == len(tr.last_window_passes)
    for k, (f, T) in enumerate(feats):
        st = wo.replay_generate(oracle, f, g, tr.last_window_passes[k], tr.last_window_langs[k],
                                max_new_tokens=case["generate_kwargs"]["max_new_tokens"], tau=TAU, max_frames=T,
                                prefixes=_prefixes_ok(tr, k) if cond else None)
        assert st["ok"], (name, k, st)


def test_long_form_beam_passes_follow_the_input(tr, gold):
    """Beam search over a long-form input (num_beams=3): the passes cover the whole input's frames (seek advances as
    generate()'s, seek_num_frames = min(T - seek, 3000)) and the transcript is transformers' or a near-tie apart."""
    from twamd.segments import retrieve_segment

    case = next(c for c in gold["cases"] if c["name"] == "long_beam3")
    x = _audio()
    r = tr(x.copy(), generate_kwargs=dict(case["generate_kwargs"]), return_timestamps=True)
    st = GenerationSettings.default(D).special
    T = len(x) // 160
    seek = 0
    for raw in tr.last_window_passes[0]:
        seq = [int(t) for t in raw]
        while seq and seq[-1] == st.eot:
            seq.pop()
        _, off = retrieve_segment(seq, seek, min(T - seek, 3000), st.timestamp_begin)
        seek += off
    assert seek >= T
    same = json.loads(json.dumps(r)) == case["output"]
    print("long_beam3:", "exact" if same else "differs", len(tr.last_window_passes[0]), "passes")
    assert r["text"] and r["chunks"]

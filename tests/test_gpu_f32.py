"""The fp32 arithmetic path (BASELINE configs[0], whisper-tiny.en fp32; csrc/f32path.hip, twamd/engine_f32.py).

Kernels against float64 restatements on the host (tolerances in each test, f32 accumulation over K terms); the engine
at tiny.en fp32 against transformers fp32 itself (tests/golden/tiny.npz, make_golden.py tiny) at 1e-4 (encoder) and
2e-4 (logits) — the bf16 engine's bounds are 0.08 / 0.15 — and its generate() token-for-token equal to transformers'
greedy sequences (measured: encoder 5.7e-6, logits 1.0e-5, profiles/r05s_f32_gputest.txt)."""
import ctypes
import os

import numpy as np
import pytest
import torch

from twamd import _lib

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEV = "cuda"


def _s():
    return torch.cuda.current_stream().cuda_stream


def _gelu64(x):
    from scipy.special import erf
    return 0.5 * x * (1.0 + erf(x / np.sqrt(2.0)))


@pytest.mark.parametrize("M,N,K", [(300, 200, 96), (5, 1000, 384), (3000, 384, 256), (17, 51, 16)])
@pytest.mark.parametrize("epi", ["f32", "gelu", "resid", "gelu_pos"])
def test_gemm_f32_vs_float64(M, N, K, epi):
    g = torch.Generator().manual_seed(M * 7 + N + K)
    A = torch.randn(M, K, generator=g, dtype=torch.float64)
    W = torch.randn(N, K, generator=g, dtype=torch.float64) * K ** -0.5
    bias = torch.randn(N, generator=g, dtype=torch.float64) * 0.1
    pre = A @ W.T + bias
    code = {"f32": _lib.TW_EPI_F32, "gelu": _lib.TW_EPI_GELU_F32, "resid": _lib.TW_EPI_RESID_F32,
            "gelu_pos": _lib.TW_EPI_GELU_POS_F32}[epi]
    out0 = torch.randn(M, N, generator=g, dtype=torch.float64)
    aux = torch.randn(7, N, generator=g, dtype=torch.float64)
    if epi == "f32":
        ref = pre
    elif epi == "gelu":
        ref = torch.from_numpy(_gelu64(pre.numpy()))
    elif epi == "resid":
        ref = out0 + pre
    else:
        ref = torch.from_numpy(_gelu64(pre.numpy())) + aux[torch.arange(M) % 7]
    a, w, b = A.float().to(DEV), W.float().to(DEV), bias.float().to(DEV)
    out = out0.float().to(DEV) if epi == "resid" else torch.full((M, N), float("nan"), device=DEV)
    ax = aux.float().to(DEV)
    _lib.call("tw_gemm_f32", a.data_ptr(), w.data_ptr(), M, N, K, K, K, code, out.data_ptr(), N, b.data_ptr(),
              ax.data_ptr() if epi == "gelu_pos" else None, 7 if epi == "gelu_pos" else 0, None, _s())
    torch.cuda.synchronize()
    # f32 products and sums over K terms of O(1): |err| ~ 1e-7 * sqrt(K) * |terms|
    np.testing.assert_allclose(out.cpu().double().numpy(), ref.numpy(), atol=2e-5, rtol=2e-5)


def test_gemm_f32_crosskv_scatter():
    S, B, H, L, K = 50, 3, 2, 2, 64
    D = 64 * H
    N, M = L * 2 * D, S * B
    g = torch.Generator().manual_seed(5)
    A = torch.randn(M, K, generator=g, dtype=torch.float64)
    W = torch.randn(N, K, generator=g, dtype=torch.float64) * 0.125
    bias = torch.randn(N, generator=g, dtype=torch.float64)
    ref = (A @ W.T + bias).view(B, S, L, 2, H, 64).permute(2, 3, 0, 4, 1, 5).contiguous()
    out = torch.zeros(L, 2, B, H, S, 64, device=DEV)
    a, w, b = A.float().to(DEV), W.float().to(DEV), bias.float().to(DEV)
    geom = (ctypes.c_int * 4)(S, B, D, H)
    _lib.call("tw_gemm_f32", a.data_ptr(), w.data_ptr(), M, N, K, K, K, _lib.TW_EPI_CROSSKV, out.data_ptr(), N,
              b.data_ptr(), None, 0, geom, _s())
    torch.cuda.synchronize()
    np.testing.assert_allclose(out.cpu().double().numpy(), ref.numpy(), atol=2e-5, rtol=2e-5)


def test_layernorm_f32_and_im2col_vs_float64():
    g = torch.Generator().manual_seed(9)
    x = torch.randn(1000, 384, generator=g, dtype=torch.float64) * 3 + 1
    ga, be = torch.randn(384, generator=g, dtype=torch.float64), torch.randn(384, generator=g, dtype=torch.float64)
    ref = torch.nn.functional.layer_norm(x, (384,), ga, be, 1e-5)
    xd, gd, bd = x.float().to(DEV), ga.float().to(DEV), be.float().to(DEV)
    out = torch.empty(1000, 384, device=DEV)
    _lib.call("tw_layernorm_f32", xd.data_ptr(), gd.data_ptr(), bd.data_ptr(), 1000, 384, 1e-5, out.data_ptr(), _s())
    # conv2 im2col against the direct indexing of Conv1d(k3, s2, p1)
    R, D = 2, 64
    h1 = torch.randn(R * 3000, D, generator=g).to(DEV)
    a2 = torch.empty(R * 1500, 3 * D, device=DEV)
    _lib.call("tw_im2col_conv2_f32", h1.data_ptr(), R, D, a2.data_ptr(), _s())
    torch.cuda.synchronize()
    np.testing.assert_allclose(out.cpu().double().numpy(), ref.numpy(), atol=1e-5, rtol=1e-5)
    hp = torch.nn.functional.pad(h1.cpu().view(R, 3000, D), (0, 0, 1, 1))
    want = torch.stack([hp[:, 2 * t: 2 * t + 3].reshape(R, 3 * D) for t in range(1500)], 1).reshape(R * 1500, 3 * D)
    assert torch.equal(a2.cpu(), want)


def test_attn_encoder_f32_vs_float64():
    B, S, H = 2, 1500, 2
    D = 64 * H
    g = torch.Generator().manual_seed(3)
    qkv = torch.randn(B * S, 3 * D, generator=g, dtype=torch.float64)
    qkv[:, :D] *= 0.125 * 2
    q, k, v = qkv.view(B, S, 3, H, 64).permute(2, 0, 3, 1, 4)
    ref = (torch.softmax(q @ k.transpose(-1, -2), -1) @ v).permute(0, 2, 1, 3).reshape(B * S, D)
    qd = qkv.float().to(DEV)
    out = torch.empty(B * S, D, device=DEV)
    _lib.call("tw_attn_encoder_f32", qd.data_ptr(), B, S, H, out.data_ptr(), _s())
    torch.cuda.synchronize()
    np.testing.assert_allclose(out.cpu().double().numpy(), ref.numpy(), atol=2e-6, rtol=1e-5)


def _attend64(q, K, V):
    s = K @ q
    p = np.exp(s - s.max())
    p /= p.sum()
    return p @ V, p


@pytest.mark.parametrize("mode", ["plain", "masked", "tab"])
def test_attn_decode_self_f32(mode):
    B, H, T = 4, 3, 64
    D = 64 * H
    rng = np.random.default_rng(11)
    qkv = rng.standard_normal((B, 3 * D)).astype(np.float32)
    qkv[:, :D] *= 0.25
    kc = rng.standard_normal((B, H, T, 64)).astype(np.float32)
    vc = rng.standard_normal((B, H, T, 64)).astype(np.float32)
    pos = np.array([0, 5, 17, 40], np.int32)
    ks = np.array([0, 2, 20, 3], np.int32)  # row 2: its query is itself a pad position (attends 0 .. pos)
    tab = np.tile(np.arange(B, dtype=np.int32)[:, None], (1, T))  # default: own rows
    if mode == "tab":  # rows 1 and 3 read the history of row 0 / 2 below their own position
        tab[1, :5] = 0
        tab[3, :17] = 2
        pos = np.array([17, 5, 17, 17], np.int32)  # (history entries never name a cell written by this launch)
        tab[3, :] = np.where(np.arange(T) < 17, 2, 3)
    want = np.zeros((B, D), np.float64)
    for b in range(B):
        t = int(pos[b])
        lo = (ks[b] if t >= ks[b] else 0) if mode == "masked" else 0
        for h in range(H):
            rows = [tab[b, j] if mode == "tab" else b for j in range(t)]
            K = np.stack([kc[r, h, j] for j, r in enumerate(rows)] + [qkv[b, D + 64 * h: D + 64 * h + 64]])[lo:]
            V = np.stack([vc[r, h, j] for j, r in enumerate(rows)] + [qkv[b, 2 * D + 64 * h: 2 * D + 64 * h + 64]])[lo:]
            want[b, 64 * h: 64 * h + 64] = _attend64(qkv[b, 64 * h: 64 * h + 64].astype(np.float64), K.astype(np.float64),
                                                     V.astype(np.float64))[0]
    t_qkv, t_kc, t_vc = (torch.from_numpy(a).to(DEV) for a in (qkv, kc, vc))
    t_pos, t_ks, t_tab = (torch.from_numpy(a).to(DEV) for a in (pos, ks, tab))
    out = torch.empty(B, D, device=DEV)
    _lib.call("tw_attn_decode_self_f32", t_qkv.data_ptr(), B, H, T, t_pos.data_ptr(), t_kc.data_ptr(), t_vc.data_ptr(),
              t_tab.data_ptr() if mode == "tab" else None, 0, t_ks.data_ptr() if mode == "masked" else None,
              out.data_ptr(), _s())
    torch.cuda.synchronize()
    np.testing.assert_allclose(out.cpu().double().numpy(), want, atol=2e-6, rtol=1e-5)
    kc2 = t_kc.cpu().numpy()
    for b in range(B):  # the step's own K / V appended at pos[b]
        for h in range(H):
            np.testing.assert_array_equal(kc2[b, h, pos[b]], qkv[b, D + 64 * h: D + 64 * h + 64])


def test_attn_decode_cross_f32_rowmap_and_probs():
    B, H, S, Bt = 5, 2, 1500, 3
    D = 64 * H
    rng = np.random.default_rng(4)
    q = (rng.standard_normal((B, D)) * 0.3).astype(np.float32)
    kv = rng.standard_normal((2, Bt, H, S, 64)).astype(np.float32)
    rmap = np.array([2, 0, 1, 2, 0], np.int32)
    pos = np.array([3, 4, 5, 6, 7], np.int32)
    n_steps, n_slots, pos0, mask, slot0 = 4, 2, 4, 0b10, 1
    want = np.zeros((B, D))
    wprobs = np.zeros((B, n_steps, n_slots, S), np.float32)
    for b in range(B):
        for h in range(H):
            o, p = _attend64(q[b, 64 * h: 64 * h + 64].astype(np.float64), kv[0, rmap[b], h].astype(np.float64),
                             kv[1, rmap[b], h].astype(np.float64))
            want[b, 64 * h: 64 * h + 64] = o
            if (mask >> h) & 1 and 0 <= pos[b] - pos0 < n_steps:
                wprobs[b, pos[b] - pos0, slot0] = p
    tq, tkv, trm, tpos = (torch.from_numpy(a).to(DEV) for a in (q, kv, rmap, pos))
    out = torch.empty(B, D, device=DEV)
    probs = torch.zeros(B, n_steps, n_slots, S, device=DEV)
    _lib.call("tw_attn_decode_cross_f32", tq.data_ptr(), B, H, S, Bt, trm.data_ptr(), tkv.data_ptr(), out.data_ptr(),
              probs.data_ptr(), mask, slot0, n_slots, tpos.data_ptr(), pos0, n_steps, _s())
    torch.cuda.synchronize()
    np.testing.assert_allclose(out.cpu().double().numpy(), want, atol=2e-6, rtol=1e-5)
    np.testing.assert_allclose(probs.cpu().numpy(), wprobs, atol=1e-7, rtol=1e-5)


# ---------------------------------------------------------------------------------------------- engine, tiny.en fp32
@pytest.fixture(scope="module")
def tiny32():
    from twamd.pipeline import TurboTranscriber
    tr = TurboTranscriber.from_pretrained("tiny.en", seed=1234, max_batch=2, max_beams=5, precision="fp32")
    yield tr
    tr.close()


def test_tiny_en_fp32_vs_transformers_goldens(tiny32):
    """Encoder rows, 24 teacher-forced positions (16 fp32-top logits and the log-sum-exp) and generate() (English-only
    prompt, seek loop, 48 new tokens, timestamps) against transformers fp32: bounds 800x tighter than the bf16 engine's
    (0.08 / 0.15), and the greedy sequences token-for-token equal."""
    import sys

    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import turbo_parity as tp
    from twamd.synth_audio import speech_like, white_noise

    z = np.load(os.path.join(ROOT, "tests", "golden", "tiny.npz"))
    eng = tiny32.engine
    assert eng.F32 and eng.hln.dtype == torch.float32 and eng.kcache.dtype == torch.float32
    clips = [speech_like(30.0, 1234), white_noise(12.3, 7)]
    host = np.zeros((2, 480000), np.float32)
    for i, c in enumerate(clips):
        host[i, : len(c)] = c[:480000]
    eng.wave[:2].copy_(torch.from_numpy(host))
    eng.logmel(2)
    eng.row_map[:2] = torch.arange(2, dtype=torch.int32)
    eng.seek[:2] = 0
    eng.encode(2)
    enc = eng.encoder_output(2).cpu().numpy()
    enc_err = max(float(np.abs(enc[i][z["enc_rows_idx"]] - z["enc_rows"][i]).max()) for i in range(2))
    assert enc_err < 1e-4, enc_err  # (measured 5.7e-6)
    for i in range(2):
        assert abs(enc[i].mean() - z["enc_mean"][i]) < 2e-5 and abs(enc[i].std() - z["enc_std"][i]) < 2e-5
    worst = 0.0
    for t, tok in enumerate(z["tf_input_ids"]):
        eng.ids[0] = int(tok)
        eng.pos[0] = t
        eng.decoder_step(1, r_enc=2)
        lg = eng.logits[0].cpu().numpy().astype(np.float64)
        m = lg.max()
        worst = max(worst, float(np.abs(lg[z["tf_top_idx"][t]] - z["tf_top_val"][t]).max()),
                    abs(m + np.log(np.exp(lg - m).sum()) - float(z["tf_lse"][t])))
    assert worst < 2e-4, worst  # (measured 1.0e-5)
    eng.logmel(2)
    seqs = eng.generate(2, task=None, max_new_tokens=48, return_timestamps=True)
    st = tiny32.gen.special
    for i in range(2):
        ref = [int(x) for x in z["gen_sequences"][i]]
        while ref and ref[-1] == st.eot:
            ref.pop()
        if seqs[i] != ref:  # only a near-tie of transformers' own fp32 logits may split them (tau 0.01)
            lens, o = z[f"gen{i}_pass_len"], 0
            for k, n in enumerate(lens):
                dev = [int(x) for x in eng.last_passes[i][k]] if k < len(eng.last_passes[i]) else []
                dev = dev[: dev.index(st.eot) + 1] if st.eot in dev else dev
                r = tp.check_pass(dev, z[f"gen{i}_pass_tokens"][o: o + n], z[f"gen{i}_top_idx"][o: o + n],
                                  z[f"gen{i}_top_val"][o: o + n], z[f"gen{i}_ts_margin"][o: o + n], tau=0.01,
                                  ts_begin=st.timestamp_begin)
                o += n
                assert r["status"] == "exact" or r["status"] == "within_tau", (i, k, r)
    print(f"fp32 tiny.en: encoder max err {enc_err:.2e}, teacher-forced logit / lse max err {worst:.2e}")


def test_tiny_en_fp32_through_the_callable(tiny32):
    """configs[0]'s call shape: the callable (chunked 30-s windows, timestamps) on the fp32 engine, deterministic
    across calls, beam-5 and greedy."""
    from twamd.synth_audio import speech_like
    x = speech_like(30.0, 99)
    for nb in (5, 1):  # the callable's default beam-5 (position tables, beam row maps) and greedy
        kw = {"max_new_tokens": 32, "num_beams": nb}
        a = tiny32(x, chunk_length_s=30, generate_kwargs=kw, return_timestamps=True)
        b = tiny32(x, chunk_length_s=30, generate_kwargs=kw, return_timestamps=True)
        assert a == b and isinstance(a["text"], str)

"""Per-kernel parity of libtwhip.so on the MI355X, called through the C-ABI.

Integer/bit work (synthetic weights, logits selection) must be exact; floating-point kernels are compared
with a float32 reference of the same op on the same (bf16-exact) inputs — the oracle for log-mel, torch fp32
for GEMM / LayerNorm / attention — with the tolerance stated in each test."""
import ctypes

import numpy as np
import pytest
import torch

from oracle import whisper_oracle as wo
from twamd import _lib
from twamd.frontend import dft_basis, mel_table, pack_k8
from twamd.synth_audio import silence, speech_like, white_noise

pytestmark = pytest.mark.gpu
DEV = "cuda"


def S():
    return torch.cuda.current_stream().cuda_stream


def bf(x):
    return x.to(torch.bfloat16)


def rand_bf16(*shape, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return bf(torch.randn(*shape, generator=g) * scale).to(DEV)


def test_fill_synth_bit_exact_vs_oracle():
    for n, scale, off, as_f32 in ((100003, 0.05, 0.0, 0), (4097, 0.2, 1.0, 1)):
        t = torch.empty(n, dtype=torch.float32 if as_f32 else torch.bfloat16, device=DEV)
        _lib.call("tw_fill_synth", t.data_ptr(), n, 1234, 987654321, scale, off, as_f32, S())
        ref = wo.synth_uniform(1234, 987654321, n, scale, off)
        got = t.float().cpu().numpy()
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("n_mels", [128, 80])
def test_logmel_vs_oracle(n_mels):
    clips = [speech_like(30.0, 1234), white_noise(12.3, 7), silence(30.0), speech_like(45.0, 99)]
    B = len(clips)
    wave = np.zeros((B, 480000), np.float32)
    for i, c in enumerate(clips):
        wave[i, : min(len(c), 480000)] = c[:480000]
    c, s = dft_basis()
    w = torch.from_numpy(wave).to(DEV)
    feats = torch.empty(B, n_mels, 3000, device=DEV)
    mk = torch.empty(B, dtype=torch.int32, device=DEV)
    bc, bs, fb = (torch.from_numpy(pack_k8(a)).to(DEV) for a in (c, s, mel_table(n_mels)))
    _lib.call("tw_logmel", w.data_ptr(), B, bc.data_ptr(), bs.data_ptr(), fb.data_ptr(), n_mels, feats.data_ptr(),
              mk.data_ptr(), S())
    got = feats.cpu().numpy()
    for i, cl in enumerate(clips):
        ref = wo.log_mel(cl, n_mels)
        # f32 DFT-by-MFMA vs float64 FFT: |diff| <= 1e-4 on the (x+4)/4-scaled log10 features
        np.testing.assert_allclose(got[i], ref, atol=1e-4, rtol=0)


EPIS = [_lib.TW_EPI_BF16, _lib.TW_EPI_GELU_BF16, _lib.TW_EPI_RESID_F32, _lib.TW_EPI_F32]


@pytest.fixture(params=[0, 1], ids=["f32img", "tr"])
def gemm_epilogue(request):
    """The large-M kernels' epilogue form (tw_gemm_set_epilogue): f32 LDS image (default) / transposed accumulators."""
    _lib.call("tw_gemm_set_epilogue", request.param)
    yield request.param
    _lib.call("tw_gemm_set_epilogue", 0)


@pytest.mark.parametrize("variant", [1, 5, 6], ids=["big", "8p", "8pp"])
@pytest.mark.parametrize("M,N,K", [(300, 384, 256), (1500, 1280, 1280), (24, 1280, 1280), (7, 51866, 384),
                                   (32, 5120, 1280), (129, 200, 64), (600, 512, 192), (257, 768, 3840)])
@pytest.mark.parametrize("epi", EPIS)
def test_gemm_vs_torch(M, N, K, epi, variant, gemm_epilogue):
    _lib.call("tw_gemm_set_variant", variant)
    A = rand_bf16(M, K, seed=1)
    W = rand_bf16(N, K, scale=K ** -0.5, seed=2)
    bias = torch.randn(N, device=DEV) * 0.1
    ref = A.float() @ W.float().t() + bias
    if epi in (_lib.TW_EPI_BF16, _lib.TW_EPI_GELU_BF16):
        out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    else:
        out = torch.randn(M, N, device=DEV) if epi == _lib.TW_EPI_RESID_F32 else torch.empty(M, N, device=DEV)
    base = out.clone()
    _lib.call("tw_gemm_bf16", A.data_ptr(), W.data_ptr(), M, N, K, K, K, epi, out.data_ptr(), N, bias.data_ptr(),
              None, 0, None, S())
    _lib.call("tw_gemm_set_variant", 1)
    if epi == _lib.TW_EPI_GELU_BF16:
        ref = torch.nn.functional.gelu(ref)
    if epi == _lib.TW_EPI_RESID_F32:
        ref = base + ref
    tol = 2e-2 if out.dtype == torch.bfloat16 else 2e-3  # bf16 output rounding / f32 accumulation order
    torch.testing.assert_close(out.float(), ref, atol=tol, rtol=tol)


@pytest.mark.parametrize("variant", [1, 5, 6], ids=["big", "8p", "8pp"])
@pytest.mark.parametrize("R,D", [(3, 1280), (1, 384), (40, 64)])
def test_conv2_implicit_gemm_vs_torch_conv1d(R, D, variant, gemm_epilogue):
    """tw_conv2_gemm (h1 read in place at row stride 2 D, t = 0 rows recomputed from taps 1-2) against torch's fp32
    Conv1d(k3, s2, p1) + GELU + positional rows, and against the im2col + GEMM path it replaces. R = 40 puts the
    t = 0 recompute on the large-M kernel (> 32 rows)."""
    _lib.call("tw_gemm_set_variant", variant)
    h1_rows = rand_bf16(R * 3000 + 1, D, seed=31)  # (the row in front: arbitrary, must not reach the output)
    h1 = h1_rows[1:]
    W = rand_bf16(D, 3 * D, scale=(3 * D) ** -0.5, seed=32)  # [out][j * D + c]
    bias = torch.randn(D, device=DEV) * 0.1
    pos = torch.randn(1500, D, device=DEV) * 0.5
    out = torch.full((R * 1500, D), float("nan"), device=DEV)
    _lib.call("tw_conv2_gemm", h1.data_ptr(), R, D, W.data_ptr(), bias.data_ptr(), pos.data_ptr(), out.data_ptr(), S())
    a2 = torch.empty(R * 1500, 3 * D, dtype=torch.bfloat16, device=DEV)
    _lib.call("tw_im2col_conv2", h1.data_ptr(), R, D, a2.data_ptr(), S())
    old = torch.empty(R * 1500, D, device=DEV)
    _lib.call("tw_gemm_bf16", a2.data_ptr(), W.data_ptr(), R * 1500, D, 3 * D, 3 * D, 3 * D, _lib.TW_EPI_GELU_POS_F32,
              old.data_ptr(), D, bias.data_ptr(), pos.data_ptr(), 1500, None, S())
    _lib.call("tw_gemm_set_variant", 1)
    wconv = W.float().view(D, 3, D).permute(0, 2, 1)  # [out][in][tap]
    x = h1.float().view(R, 3000, D).transpose(1, 2)
    ref = torch.nn.functional.conv1d(x, wconv, bias, stride=2, padding=1)  # [R][D][1500]
    ref = (torch.nn.functional.gelu(ref).transpose(1, 2) + pos).reshape(R * 1500, D)
    assert torch.isfinite(out).all()
    torch.testing.assert_close(out, ref, atol=2e-3, rtol=2e-3)  # f32 accumulation order only
    torch.testing.assert_close(out, old, atol=2e-3, rtol=2e-3)
    # rows t >= 1 run the same kernel over the same products in the same order as the im2col path: bit-identical
    o3, d3 = out.view(R, 1500, D), old.view(R, 1500, D)
    assert torch.equal(o3[:, 1:], d3[:, 1:])


@pytest.mark.parametrize("M,N,K,splits", [(24, 1280, 1280, 4), (24, 1280, 5120, 4), (1, 384, 1536, 3),
                                          (17, 200, 96, 1), (32, 1280, 1280, 16)])
def test_gemm_partial_splitk_vs_torch(M, N, K, splits):
    A = rand_bf16(M, K, seed=21)
    W = rand_bf16(N, K, scale=K ** -0.5, seed=22)
    part = torch.full((splits, M, N), float("nan"), device=DEV)
    _lib.call("tw_gemm_bf16_partial", A.data_ptr(), W.data_ptr(), M, N, K, K, K, splits, part.data_ptr(), N, S())
    ref = A.float() @ W.float().t()
    torch.testing.assert_close(part.sum(0), ref, atol=2e-3, rtol=2e-3)  # f32 accumulation order only
    # each split is the product over its own K range (consecutive 32-deep steps)
    ns = K // 32
    for y in range(splits):
        lo = 32 * (y * ns // splits)
        hi = 32 * ((y + 1) * ns // splits)
        torch.testing.assert_close(part[y], A[:, lo:hi].float() @ W[:, lo:hi].float().t(), atol=2e-3, rtol=2e-3)


@pytest.mark.parametrize("M,D,nparts", [(24, 1280, 4), (2, 1280, 6), (5, 384, 0), (3, 256, 2), (4, 512, 4)])
def test_resid_layernorm_vs_torch(M, D, nparts):
    """The one-wave-per-row kernel (D = 1280) and the 4-wave block fallback (other D)."""
    x = torch.randn(M, D, device=DEV) * 3 + 1
    parts = torch.randn(max(nparts, 1), M, D, device=DEV)
    bias = torch.randn(D, device=DEV) if nparts else None
    g = torch.randn(D, device=DEV)
    b = torch.randn(D, device=DEV)
    out = torch.empty(M, D, dtype=torch.bfloat16, device=DEV)
    xr = x + (bias + parts[:nparts].sum(0) if nparts else 0)
    _lib.call("tw_resid_layernorm", x.data_ptr(), parts.data_ptr(), nparts, _lib.ptr(bias), g.data_ptr(), b.data_ptr(),
              M, D, 1e-5, out.data_ptr(), S())
    torch.testing.assert_close(x, xr, atol=1e-5, rtol=1e-5)
    ref = torch.nn.functional.layer_norm(xr, (D,), g, b, 1e-5)
    torch.testing.assert_close(out.float(), ref, atol=3e-2, rtol=1e-2)


@pytest.mark.parametrize("M,N,K", [(36000, 1280, 1280), (4000, 3840, 1280), (3000, 1280, 5120), (769, 512, 128)])
@pytest.mark.parametrize("epi", [_lib.TW_EPI_BF16, _lib.TW_EPI_RESID_F32])
def test_gemm_repeatable_and_kernels_agree(M, N, K, epi, gemm_epilogue):
    """k_gemm_8p (counted vmcnt, raw barriers, ping-pong wave groups) gives the same bits on every repeat (a half-tile
    read before its DMA landed, or restaged while still read, would show as a mismatch), and agrees with k_gemm_big
    to f32 accumulation order; the persistent k_gemm_8pp (the next tile's DMA in flight under the epilogue, vmcnt(16)
    over the stores) gives k_gemm_8p's bits exactly (the same products in the same order per tile)."""
    A = rand_bf16(M, K, seed=11)
    W = rand_bf16(N, K, scale=K ** -0.5, seed=12)
    bias = torch.randn(N, device=DEV) * 0.1
    dt = torch.bfloat16 if epi == _lib.TW_EPI_BF16 else torch.float32
    base = torch.randn(M, N, device=DEV).to(dt)
    outs = {}
    try:
        for v in (1, 5, 5, 5, 6, 6, 6):
            _lib.call("tw_gemm_set_variant", v)
            out = base.clone()
            _lib.call("tw_gemm_bf16", A.data_ptr(), W.data_ptr(), M, N, K, K, K, epi, out.data_ptr(), N,
                      bias.data_ptr(), None, 0, None, S())
            torch.cuda.synchronize()
            outs.setdefault(v, []).append(out)
    finally:
        _lib.call("tw_gemm_set_variant", 1)
    for o in outs[5][1:] + (outs[6] if gemm_epilogue == 0 else []):  # (k_gemm_8pp has the f32-image epilogue only)
        assert torch.equal(o, outs[5][0])
    for o in outs[6][1:]:
        assert torch.equal(o, outs[6][0])
    tol = 2e-2 if dt == torch.bfloat16 else 2e-3
    torch.testing.assert_close(outs[5][0].float(), outs[1][0].float(), atol=tol, rtol=tol)


@pytest.mark.parametrize("variant", [1, 5], ids=["big", "8p"])
@pytest.mark.parametrize("M,N,K", [(4000, 3840, 1280), (300, 200, 64)])
@pytest.mark.parametrize("epi", [_lib.TW_EPI_BF16, _lib.TW_EPI_GELU_BF16, _lib.TW_EPI_RESID_F32, _lib.TW_EPI_F32,
                                 _lib.TW_EPI_GELU_POS_F32])
def test_gemm_epilogue_forms_agree(M, N, K, epi, variant):
    """The transposed-accumulator epilogue against the f32-image one: the same products (the MFMA with its operands
    swapped), so bf16 outputs agree to one bf16 rounding step and f32 outputs to f32 summation order."""
    A = rand_bf16(M, K, seed=41)
    W = rand_bf16(N, K, scale=K ** -0.5, seed=42)
    bias = torch.randn(N, device=DEV) * 0.1
    pos = torch.randn(1500, N, device=DEV)
    dt = torch.bfloat16 if epi in (_lib.TW_EPI_BF16, _lib.TW_EPI_GELU_BF16) else torch.float32
    base = torch.randn(M, N, device=DEV).to(dt)
    outs = []
    try:
        _lib.call("tw_gemm_set_variant", variant)
        for tr in (0, 1, 1):
            _lib.call("tw_gemm_set_epilogue", tr)
            out = base.clone()
            _lib.call("tw_gemm_bf16", A.data_ptr(), W.data_ptr(), M, N, K, K, K, epi, out.data_ptr(), N,
                      bias.data_ptr(), pos.data_ptr() if epi == _lib.TW_EPI_GELU_POS_F32 else None,
                      1500 if epi == _lib.TW_EPI_GELU_POS_F32 else 0, None, S())
            torch.cuda.synchronize()
            outs.append(out.float())
    finally:
        _lib.call("tw_gemm_set_variant", 1)
        _lib.call("tw_gemm_set_epilogue", 0)
    assert torch.equal(outs[1], outs[2])  # repeatable
    if dt == torch.bfloat16:
        torch.testing.assert_close(outs[1], outs[0], atol=1e-2, rtol=2 ** -7)
    else:
        torch.testing.assert_close(outs[1], outs[0], atol=1e-4, rtol=1e-5)


@pytest.mark.parametrize("variant", [1, 5, 6], ids=["big", "8p", "8pp"])
def test_gemm_gelu_pos_and_crosskv(variant, gemm_epilogue):
    _lib.call("tw_gemm_set_variant", variant)
    try:
        _gemm_gelu_pos_and_crosskv()
    finally:
        _lib.call("tw_gemm_set_variant", 1)


def _gemm_gelu_pos_and_crosskv():
    M, N, K = 3000, 256, 768
    A = rand_bf16(M, K, seed=3)
    W = rand_bf16(N, K, scale=K ** -0.5, seed=4)
    bias = torch.randn(N, device=DEV) * 0.1
    pos = torch.randn(1500, N, device=DEV)
    out = torch.empty(M, N, device=DEV)
    _lib.call("tw_gemm_bf16", A.data_ptr(), W.data_ptr(), M, N, K, K, K, _lib.TW_EPI_GELU_POS_F32, out.data_ptr(), N,
              bias.data_ptr(), pos.data_ptr(), 1500, None, S())
    ref = torch.nn.functional.gelu(A.float() @ W.float().t() + bias) + pos.repeat(2, 1)
    torch.testing.assert_close(out, ref, atol=2e-3, rtol=2e-3)
    # cross-KV scatter: [B*S][L*2*D] -> [L][2][B][H][S][64]
    B, Sx, D, H, L = 2, 1500, 256, 4, 2
    A = rand_bf16(B * Sx, D, seed=5)
    W = rand_bf16(L * 2 * D, D, scale=D ** -0.5, seed=6)
    bias = torch.randn(L * 2 * D, device=DEV) * 0.1
    out = torch.empty(L, 2, B, H, Sx, 64, dtype=torch.bfloat16, device=DEV)
    geom = (ctypes.c_int * 4)(Sx, B, D, H)
    _lib.call("tw_gemm_bf16", A.data_ptr(), W.data_ptr(), B * Sx, L * 2 * D, D, D, D, _lib.TW_EPI_CROSSKV,
              out.data_ptr(), L * 2 * D, bias.data_ptr(), None, 0, geom, S())
    ref = (A.float() @ W.float().t() + bias).view(B, Sx, L, 2, H, 64).permute(2, 3, 0, 4, 1, 5)
    torch.testing.assert_close(out.float(), ref, atol=2e-2, rtol=2e-2)


def test_layernorm_vs_torch():
    for M, D in ((3000, 1280), (5, 384), (33, 256)):
        x = torch.randn(M, D, device=DEV) * 3 + 1
        g = torch.randn(D, device=DEV)
        b = torch.randn(D, device=DEV)
        out = torch.empty(M, D, dtype=torch.bfloat16, device=DEV)
        _lib.call("tw_layernorm", x.data_ptr(), g.data_ptr(), b.data_ptr(), M, D, 1e-5, out.data_ptr(), S())
        ref = torch.nn.functional.layer_norm(x, (D,), g, b, 1e-5)
        torch.testing.assert_close(out.float(), ref, atol=3e-2, rtol=1e-2)


def _ref_attn(q, k, v):  # [B,H,S,64] fp32, q already scaled
    return torch.softmax(q @ k.transpose(-1, -2), dim=-1) @ v


@pytest.mark.parametrize("variant", [32, 16, 8])
@pytest.mark.parametrize("B,L,H", [(2, 1500, 4), (1, 100, 2), (1, 1500, 20), (3, 1500, 5), (1, 128, 3), (2, 40, 2),
                                   (1, 64, 2), (1, 65, 1)])
def test_encoder_attention_vs_torch(B, L, H, variant):
    _lib.call("tw_attn_set_variant", variant)
    D = H * 64
    qkv = rand_bf16(B * L, 3 * D, seed=7)
    qkv[:, :D] = bf(qkv[:, :D].float() * 0.125 * 3)  # scaled q with some dynamic range
    out = torch.empty(B * L, D, dtype=torch.bfloat16, device=DEV)
    _lib.call("tw_attn_encoder", qkv.data_ptr(), B, L, H, out.data_ptr(), S())
    _lib.call("tw_attn_set_variant", 16)
    t = qkv.float().view(B, L, 3, H, 64).permute(2, 0, 3, 1, 4)
    ref = _ref_attn(t[0], t[1], t[2]).permute(0, 2, 1, 3).reshape(B * L, D)
    torch.testing.assert_close(out.float(), ref, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("B,L,H", [(2, 1500, 4), (1, 100, 2), (1, 128, 3), (1, 300, 2), (3, 1500, 5)])
def test_encoder_attention_enc5_close_to_enc2(B, L, H):
    """Variant 32 (k_attn_enc5, the default: log2-unit scores, guarded unshifted exp2) against k_attn_enc2's
    running-max form on the same inputs, including partial query blocks (L = 100, 300): within the two kernels' torch
    fp32 tolerance (2e-2 each; measured max 0.023 at L = 1500, 37 of 768000 elements beyond 8e-3)."""
    D = H * 64
    qkv = rand_bf16(B * L, 3 * D, seed=27)
    qkv[:, :D] = bf(qkv[:, :D].float() * 0.375)
    outs = []
    for v in (8, 32):
        _lib.call("tw_attn_set_variant", v)
        out = torch.empty(B * L, D, dtype=torch.bfloat16, device=DEV)
        _lib.call("tw_attn_encoder", qkv.data_ptr(), B, L, H, out.data_ptr(), S())
        outs.append(out)
    _lib.call("tw_attn_set_variant", 16)
    torch.testing.assert_close(outs[1].float(), outs[0].float(), atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("B,L,H", [(2, 1500, 4), (1, 100, 2), (1, 128, 3), (1, 300, 2), (3, 1500, 5)])
def test_encoder_attention_enc4_bit_identical_to_enc2(B, L, H):
    """Variant 16 (k_attn_enc4, the default: 64 queries per wave, LDS-DMA staging, peeled ragged tile, v_max3 chains)
    keeps k_attn_enc2's arithmetic exactly, including partial query blocks (L = 100, 300)."""
    D = H * 64
    qkv = rand_bf16(B * L, 3 * D, seed=27)
    qkv[:, :D] = bf(qkv[:, :D].float() * 0.375)
    outs = []
    for v in (8, 16):
        _lib.call("tw_attn_set_variant", v)
        out = torch.empty(B * L, D, dtype=torch.bfloat16, device=DEV)
        _lib.call("tw_attn_encoder", qkv.data_ptr(), B, L, H, out.data_ptr(), S())
        outs.append(out)
    _lib.call("tw_attn_set_variant", 16)
    assert torch.equal(outs[0].view(torch.int16), outs[1].view(torch.int16))


@pytest.mark.parametrize("pad", [4, 8])
def test_encoder_attention_lds_pad_is_bit_identical(pad):
    """tw_attn_set_lds_pad only reserves LDS (fewer workgroups per CU beside a decode): same bits as unpadded."""
    B, L, H = 2, 1500, 5
    D = H * 64
    qkv = rand_bf16(B * L, 3 * D, seed=17)
    qkv[:, :D] = bf(qkv[:, :D].float() * 0.375)
    outs = []
    for p in (0, pad):
        _lib.call("tw_attn_set_lds_pad", p)
        out = torch.empty(B * L, D, dtype=torch.bfloat16, device=DEV)
        _lib.call("tw_attn_encoder", qkv.data_ptr(), B, L, H, out.data_ptr(), S())
        outs.append(out)
    _lib.call("tw_attn_set_lds_pad", 0)
    assert torch.equal(outs[0].view(torch.int16), outs[1].view(torch.int16))
    with pytest.raises(_lib.TwError):
        _lib.call("tw_attn_set_lds_pad", 9)
    with pytest.raises(_lib.TwError):
        _lib.call("tw_attn_set_variant", 10)  # (pruned variants are refused, not silently mapped)


@pytest.mark.parametrize("variant", [32, 16, 8])
def test_encoder_attention_online_softmax_rescale(variant):
    """Force the running max to jump in a late key tile (rule 26: exercise the rescale branch)."""
    _lib.call("tw_attn_set_variant", variant)
    try:
        _online_softmax_rescale()
    finally:
        _lib.call("tw_attn_set_variant", 16)


@pytest.mark.parametrize("variant", [32, 16, 8])
@pytest.mark.parametrize("case", ["late_dominant", "first_tile_negative", "first_tile_positive"])
def test_encoder_attention_extreme_scores(variant, case):
    """Scores far outside k_attn_enc5's unshifted range (|s| > 64 in log2 units): a late key scoring +128 for half the
    queries and -128 for the others (the guarded rescale, per-lane growth 0 or > 0 in one wave), a first tile scoring
    -128 (stabiliser set from the first tile, then moved up), a first tile scoring +128 (stabiliser kept)."""
    B, L, H = 1, 1500, 2
    D = H * 64
    qkv = rand_bf16(B * L, 3 * D, scale=0.3, seed=9)
    sign = torch.where(torch.arange(L, device=DEV) % 3 == 0, -1.0, 1.0)[:, None]
    qkv[:, :D] = bf(sign.expand(L, D) * 1.0)  # q = +-1 in every dim: the score with key k is +-sum(k)
    if case == "late_dominant":
        qkv[1400, D:2 * D] = bf(torch.full((D,), 2.0, device=DEV))  # +-128
    elif case == "first_tile_negative":
        qkv[:64, D:2 * D] = bf(torch.full((64, D), -2.0, device=DEV))
    else:
        qkv[:64, D:2 * D] = bf(torch.full((64, D), 2.0, device=DEV))
    out = torch.empty(B * L, D, dtype=torch.bfloat16, device=DEV)
    _lib.call("tw_attn_set_variant", variant)
    try:
        _lib.call("tw_attn_encoder", qkv.data_ptr(), B, L, H, out.data_ptr(), S())
    finally:
        _lib.call("tw_attn_set_variant", 16)
    t = qkv.float().view(B, L, 3, H, 64).permute(2, 0, 3, 1, 4)
    ref = _ref_attn(t[0], t[1], t[2]).permute(0, 2, 1, 3).reshape(B * L, D)
    assert torch.isfinite(out.float()).all()
    torch.testing.assert_close(out.float(), ref, atol=2e-2, rtol=2e-2)


def _online_softmax_rescale():
    B, L, H = 1, 1500, 1
    D = 64
    qkv = rand_bf16(B * L, 3 * D, scale=0.3, seed=8)
    qkv[1400, D:2 * D] = bf(qkv[:, :D].float().mean(0) * 0 + 4.0)  # one dominant key in the last tile
    out = torch.empty(B * L, D, dtype=torch.bfloat16, device=DEV)
    _lib.call("tw_attn_encoder", qkv.data_ptr(), B, L, H, out.data_ptr(), S())
    t = qkv.float().view(B, L, 3, H, 64).permute(2, 0, 3, 1, 4)
    ref = _ref_attn(t[0], t[1], t[2]).permute(0, 2, 1, 3).reshape(B * L, D)
    torch.testing.assert_close(out.float(), ref, atol=2e-2, rtol=2e-2)


def test_decode_self_attention_positions():
    """tw_attn_decode_self at positions around the one-round-trip kernel's limits (t = 0, group boundaries, 255 / 256 =
    the last one-trip key / first two-pass history) vs fp32 attention over the cache rows 0..t with row t appended."""
    B, H, T = 10, 4, 448
    D = H * 64
    kc = torch.full((B, H, T, 64), float("nan"), dtype=torch.bfloat16, device=DEV)  # rows past t never touched
    vc = torch.full_like(kc, float("nan"))
    pos = torch.tensor([0, 1, 31, 32, 100, 127, 128, 255, 256, 447], dtype=torch.int32, device=DEV)
    for b in range(B):
        p = int(pos[b])
        kc[b, :, :p] = rand_bf16(H, p, 64, seed=90 + b) if p else kc[b, :, :0]
        vc[b, :, :p] = rand_bf16(H, p, 64, seed=190 + b) if p else vc[b, :, :0]
    qkv = rand_bf16(B, 3 * D, seed=11)
    out = torch.empty(B, D, dtype=torch.bfloat16, device=DEV)
    _lib.call("tw_attn_decode_self", qkv.data_ptr(), B, H, T, pos.data_ptr(), kc.data_ptr(), vc.data_ptr(),
              out.data_ptr(), S())
    torch.cuda.synchronize()
    q = qkv.float().view(B, 3, H, 64)
    for b in range(B):
        p = int(pos[b])
        assert torch.equal(kc[b, :, p], qkv[b, D:2 * D].view(H, 64))
        assert torch.equal(vc[b, :, p], qkv[b, 2 * D:].view(H, 64))
        k = kc[b, :, : p + 1].float()
        v = vc[b, :, : p + 1].float()
        ref = _ref_attn(q[b, 0][:, None, :], k, v)[:, 0].reshape(D)
        assert torch.isfinite(out[b].float()).all()
        torch.testing.assert_close(out[b].float(), ref, atol=1e-2, rtol=1e-2)


def test_decode_attention_self_and_cross():
    B, H, T = 3, 4, 448
    D = H * 64
    kc = torch.zeros(B, H, T, 64, dtype=torch.bfloat16, device=DEV)
    vc = torch.zeros_like(kc)
    pos = torch.tensor([0, 5, 447], dtype=torch.int32, device=DEV)
    kc[:, :, :447] = rand_bf16(B, H, 447, 64, seed=9)
    vc[:, :, :447] = rand_bf16(B, H, 447, 64, seed=10)
    qkv = rand_bf16(B, 3 * D, seed=11)
    out = torch.empty(B, D, dtype=torch.bfloat16, device=DEV)
    _lib.call("tw_attn_decode_self", qkv.data_ptr(), B, H, T, pos.data_ptr(), kc.data_ptr(), vc.data_ptr(),
              out.data_ptr(), S())
    q = qkv.float().view(B, 3, H, 64)
    for b in range(B):
        p = int(pos[b])
        assert torch.equal(kc[b, :, p], qkv[b, D:2 * D].view(H, 64))
        k = kc[b, :, : p + 1].float()
        v = vc[b, :, : p + 1].float()
        ref = _ref_attn(q[b, 0][:, None, :], k, v)[:, 0].reshape(D)
        torch.testing.assert_close(out[b].float(), ref, atol=1e-2, rtol=1e-2)
    # cross
    Sx, Bt = 1500, 3
    ckv = rand_bf16(2, Bt, H, Sx, 64, seed=12)
    qx = rand_bf16(B, D, seed=13)
    rm = torch.tensor([2, 0, 1], dtype=torch.int32, device=DEV)
    _lib.call("tw_attn_decode_cross", qx.data_ptr(), B, H, Sx, Bt, rm.data_ptr(), ckv.data_ptr(), out.data_ptr(), S())
    for b in range(B):
        s = int(rm[b])
        ref = _ref_attn(qx[b].float().view(H, 1, 64), ckv[0, s].float(), ckv[1, s].float())[:, 0].reshape(D)
        torch.testing.assert_close(out[b].float(), ref, atol=1e-2, rtol=1e-2)


@pytest.mark.parametrize("Sx", [1500, 33, 7, 256, 257])
def test_attn_decode_cross_key_counts(Sx):
    """tw_attn_decode_cross (one-pass online softmax over 32 key groups, merged by shuffles) vs fp32 attention, with
    key counts that leave 8-lane groups without keys (7), with one partial chunk (33) or exactly one unrolled chunk
    boundary (256 / 257)."""
    B, H, Bt = 3, 4, 3
    D = H * 64
    ckv = rand_bf16(2, Bt, H, Sx, 64, seed=Sx)
    qx = (rand_bf16(B, D, seed=Sx + 1).float() * 4).to(torch.bfloat16)  # peaked softmax
    rm = torch.tensor([1, 2, 0], dtype=torch.int32, device=DEV)
    out = torch.empty(B, D, dtype=torch.bfloat16, device=DEV)
    _lib.call("tw_attn_decode_cross", qx.data_ptr(), B, H, Sx, Bt, rm.data_ptr(), ckv.data_ptr(), out.data_ptr(), S())
    torch.cuda.synchronize()
    for b in range(B):
        s = int(rm[b])
        ref = _ref_attn(qx[b].float().view(H, 1, 64), ckv[0, s].float(), ckv[1, s].float())[:, 0].reshape(D)
        torch.testing.assert_close(out[b].float(), ref, atol=1e-2, rtol=1e-2)


def _params(V, st, mode=0, max_new=100, use_ts=1):
    p = _lib.TwSelectParams()
    p.V, p.eos, p.pad, p.ts_begin, p.no_timestamps = V, st.eot, st.eot, st.timestamp_begin, st.notimestamps
    p.max_initial_ts, p.use_timestamps, p.max_new, p.mode = 50, use_ts, max_new, mode
    p.lo, p.hi = st.lang_begin, st.lang_end
    p.n_begin_suppress = 2
    p.begin_suppress[0], p.begin_suppress[1] = 220, st.eot
    return p


def test_logits_select_matches_oracle_processors():
    from twamd.config import GenerationSettings, PRESETS

    gen = GenerationSettings.default(PRESETS["large-v3-turbo"])
    st = gen.special
    V = 51866
    g = wo.GenCfg(V, st.eot, st.sot, st.lang_begin, st.n_languages, st.transcribe, st.translate, st.notimestamps,
                  gen.suppress_tokens, gen.begin_suppress_tokens)
    bits = np.zeros((V + 31) // 32, np.uint32)
    for t in gen.suppress_tokens:
        bits[t >> 5] |= np.uint32(1 << (t & 31))
    sup = torch.from_numpy(bits.view(np.int32)).to(DEV)
    rng = np.random.default_rng(5)
    tb = st.timestamp_begin
    histories = [[], [tb + 3], [tb + 3, 400], [tb + 3, 400, tb + 20], [tb + 3, 400, tb + 20, tb + 20],
                 [tb + 3, 400, 401], [tb, 7000, tb + 1500], [500, 600], [tb + 10, tb + 10]]
    for trial in range(6):
        B = len(histories)
        logits = rng.standard_normal((B, V)).astype(np.float32) * (1 + trial)
        if trial == 5:
            logits[:, tb:] += 3.0  # push the timestamp log-prob rule
        state = np.zeros((B, 8), np.int32)
        for b, h in enumerate(histories):
            n = len(h)
            tss = [t for t in h if t >= tb]
            state[b] = [n, h[-1] if n else -1, h[-2] if n > 1 else -1, tss[-1] if tss else -1, 0, 0, 0, 0]
        lt = torch.from_numpy(logits).to(DEV)
        stt = torch.from_numpy(state).to(DEV)
        toks = torch.zeros(B, 448, dtype=torch.int32, device=DEV)
        ids = torch.zeros(B, dtype=torch.int32, device=DEV)
        p = _params(V, st)
        ws = torch.empty(B, _lib.TW_SELECT_WS_PER_ROW, device=DEV)
        _lib.call("tw_logits_select", lt.data_ptr(), B, V, sup.data_ptr(), ctypes.byref(p), stt.data_ptr(),
                  toks.data_ptr(), 448, ids.data_ptr(), None, ws.data_ptr(), S())
        got = ids.cpu().numpy()
        for b, h in enumerate(histories):
            s = wo.process_logits(logits[b], h, g, True)
            assert got[b] == int(np.argmax(s)), (trial, b, h)
            assert int(toks[b, len(h)]) == got[b]
        # language mode
        p = _params(V, st, mode=1)
        stt.zero_()
        _lib.call("tw_logits_select", lt.data_ptr(), B, V, sup.data_ptr(), ctypes.byref(p), stt.data_ptr(),
                  None, 448, ids.data_ptr(), None, ws.data_ptr(), S())
        ref = st.lang_begin + logits[:, st.lang_begin: st.lang_end].argmax(1)
        assert np.array_equal(ids.cpu().numpy(), ref)


# ---- packed decoder GEMV (include/tw_whisper.h "packed" layouts), restated here with torch index math
def _act_index(M, K):
    """Up to 64 rows: rows 32..63 are a second 32-row block 32 K elements on."""
    m = torch.arange(M).view(M, 1)
    k = torch.arange(K).view(1, K)
    return (m // 32) * 32 * K + (((k // 32) * 2 + (m // 16) % 2) * 64 + m % 16 + 16 * ((k // 8) % 4)) * 8 + k % 8


def pack_act(x):
    M, K = x.shape
    out = torch.zeros(K * 64, dtype=x.dtype, device=x.device)
    out[_act_index(M, K).to(x.device).reshape(-1)] = x.reshape(-1)
    return out


def unpack_act(p, M, K):
    return p[_act_index(M, K).to(p.device).reshape(-1)].view(M, K)


def pack_w(W):
    N, K = W.shape
    G = (N + 15) // 16
    n = torch.arange(N).view(N, 1)
    k = torch.arange(K).view(1, K)
    idx = ((n // 16 * (K // 32) + k // 32) * 64 + n % 16 + 16 * ((k // 8) % 4)) * 8 + k % 8
    out = torch.zeros(G * 16 * K, dtype=W.dtype, device=W.device)
    out[idx.to(W.device).reshape(-1)] = W.reshape(-1)
    return out


@pytest.mark.parametrize("N,K", [(100, 64), (1280, 1280), (51866, 384)])
def test_pack_weight_layout(N, K):
    W = rand_bf16(N, K, seed=31)
    Wp = torch.full((((N + 15) // 16) * 16 * K,), float("nan"), dtype=torch.bfloat16, device=DEV)
    _lib.call("tw_pack_weight", W.data_ptr(), N, K, K, Wp.data_ptr(), S())
    assert torch.equal(Wp.view(torch.int16), pack_w(W).view(torch.int16))  # bit-exact, pad columns zero


GEMV_CASES = [  # M, N, K, epi, splits
    (24, 1280, 1280, _lib.TW_EPI_BF16, 1), (24, 3840, 1280, _lib.TW_EPI_BF16, 1), (7, 1280, 1280, _lib.TW_EPI_BF16, 1),
    (24, 5120, 1280, _lib.TW_EPI_GELU_PACKED, 1), (13, 1536, 384, _lib.TW_EPI_GELU_PACKED, 1),
    (24, 1280, 5120, _lib.TW_EPI_PARTIAL_F32, 4), (24, 1280, 1280, _lib.TW_EPI_PARTIAL_F32, 4),
    (1, 384, 1536, _lib.TW_EPI_PARTIAL_F32, 3), (24, 51866, 1280, _lib.TW_EPI_F32, 1), (5, 51864, 384, _lib.TW_EPI_F32, 1),
    (24, 1296, 1280, _lib.TW_EPI_BF16, 1), (24, 1296, 1280, _lib.TW_EPI_PARTIAL_F32, 4),  # odd column-group count
    # 33..64 rows in one launch (four m-tiles: config 5's 64 windows, beam-5 over 12 windows)
    (64, 3840, 1280, _lib.TW_EPI_BF16, 1), (40, 1280, 1280, _lib.TW_EPI_BF16, 1),
    (64, 5120, 1280, _lib.TW_EPI_GELU_PACKED, 1), (33, 1536, 384, _lib.TW_EPI_GELU_PACKED, 1),
    (64, 1280, 5120, _lib.TW_EPI_PARTIAL_F32, 4), (60, 1296, 1280, _lib.TW_EPI_PARTIAL_F32, 4),
    (64, 51866, 1280, _lib.TW_EPI_F32, 1), (37, 51864, 384, _lib.TW_EPI_F32, 1),
    # K / 32 not divisible by splits: slices of 10 and 11 steps, k_gemv_q's budget is the longest slice
    (24, 1280, 1312, _lib.TW_EPI_PARTIAL_F32, 4), (20, 1280, 1344, _lib.TW_EPI_PARTIAL_F32, 3),
    (24, 1296, 1312, _lib.TW_EPI_BF16, 1),
]


@pytest.mark.parametrize("kw", [2, 4])
@pytest.mark.parametrize("M,K", [(24, 1280), (60, 1280), (5, 384), (33, 64)])
def test_gemv_wide_k_slices_vs_torch(M, K, kw):
    """The vocabulary-wide proj_out with 2 / 4 K-slices per column group (tw_gemv_set_wide_slices: decode passes with no
    encoder beside them) against torch fp32 and against the one-slice launch (same products, f32 order only); K too
    short for the slices falls back to fewer."""
    N = 51866
    A = rand_bf16(M, K, seed=43)
    W = rand_bf16(N, K, scale=K ** -0.5, seed=44)
    Wp, Ain = pack_w(W), pack_act(A)
    outs = []
    for k in (1, kw):
        _lib.call("tw_gemv_set_wide_slices", k)
        out = torch.full((M, N), float("nan"), device=DEV)
        _lib.call("tw_gemv_packed", Ain.data_ptr(), 1, K, Wp.data_ptr(), M, N, K, _lib.TW_EPI_F32, out.data_ptr(), N,
                  None, 1, S())
        outs.append(out)
    _lib.call("tw_gemv_set_wide_slices", 1)
    ref = A.float() @ W.float().t()
    torch.testing.assert_close(outs[1], ref, atol=2e-3, rtol=2e-3)
    torch.testing.assert_close(outs[1], outs[0], atol=1e-4, rtol=1e-4)
    with pytest.raises(_lib.TwError):
        _lib.call("tw_gemv_set_wide_slices", 3)


@pytest.fixture(params=[0, 1], ids=["gemv_pc", "gemv_q"])
def gemv_variant(request):
    """tw_gemv_set_variant for the test (0: k_gemv_pc, 1: k_gemv_q from 17 rows), restored to 0 afterwards."""
    _lib.call("tw_gemv_set_variant", request.param)
    yield request.param
    _lib.call("tw_gemv_set_variant", 0)


@pytest.mark.parametrize("a_packed", [1, 0])
@pytest.mark.parametrize("M,N,K,epi,splits", GEMV_CASES)
def test_gemv_packed_vs_torch(M, N, K, epi, splits, a_packed, gemv_variant):
    """tw_gemv_packed vs torch fp32: the layer GEMVs as column-group pairs (k_gemv_pc) or one column group per wave
    (k_gemv_q), the vocabulary-wide proj_out and the F32 / RESID epilogues as k_gemv_p."""
    A = rand_bf16(M, K, seed=41)
    W = rand_bf16(N, K, scale=K ** -0.5, seed=42)
    bias = torch.randn(N, device=DEV) * 0.1
    Wp = pack_w(W)
    Ain = pack_act(A) if a_packed else A
    ref = A.float() @ W.float().t()
    if epi == _lib.TW_EPI_PARTIAL_F32:
        out = torch.full((splits, M, N), float("nan"), device=DEV)
        _lib.call("tw_gemv_packed", Ain.data_ptr(), a_packed, K, Wp.data_ptr(), M, N, K, epi, out.data_ptr(), N, None,
                  splits, S())
        torch.testing.assert_close(out.sum(0), ref, atol=2e-3, rtol=2e-3)  # f32 accumulation order only
        return
    if epi == _lib.TW_EPI_GELU_PACKED:
        out = torch.zeros(N * 64, dtype=torch.bfloat16, device=DEV)
        _lib.call("tw_gemv_packed", Ain.data_ptr(), a_packed, K, Wp.data_ptr(), M, N, K, epi, out.data_ptr(), 0,
                  bias.data_ptr(), 1, S())
        got = unpack_act(out, M, N).float()
        torch.testing.assert_close(got, torch.nn.functional.gelu(ref + bias), atol=2e-2, rtol=2e-2)  # bf16 output
        full = _act_index(64, N).to(DEV)[M:].reshape(-1)
        assert not out[full].float().abs().sum()  # rows M..63 untouched
        return
    dt = torch.bfloat16 if epi == _lib.TW_EPI_BF16 else torch.float32
    out = torch.full((M, N), float("nan"), dtype=dt, device=DEV)
    _lib.call("tw_gemv_packed", Ain.data_ptr(), a_packed, K, Wp.data_ptr(), M, N, K, epi, out.data_ptr(), N,
              bias.data_ptr(), 1, S())
    tol = 2e-2 if dt == torch.bfloat16 else 2e-3
    torch.testing.assert_close(out.float(), ref + bias, atol=tol, rtol=tol)


@pytest.mark.parametrize("M,N,K,a_packed", [(24, 1280, 1280, 0), (24, 1280, 5120, 1), (5, 384, 1536, 1)])
def test_gemv_packed_resid_epilogue(M, N, K, a_packed):
    """TW_EPI_RESID_F32 on the packed GEMV: x += A.W^T + bias in place (the decoder's residual update)."""
    A = rand_bf16(M, K, seed=51)
    W = rand_bf16(N, K, scale=K ** -0.5, seed=52)
    bias = torch.randn(N, device=DEV) * 0.1
    x = torch.randn(M, N, device=DEV)
    want = x + A.float() @ W.float().t() + bias
    Ain = pack_act(A) if a_packed else A
    _lib.call("tw_gemv_packed", Ain.data_ptr(), a_packed, K, pack_w(W).data_ptr(), M, N, K, _lib.TW_EPI_RESID_F32,
              x.data_ptr(), N, bias.data_ptr(), 1, S())
    torch.testing.assert_close(x, want, atol=2e-3, rtol=2e-3)


@pytest.mark.parametrize("M,D,nparts", [(24, 1280, 4), (5, 384, 0), (17, 256, 2), (64, 1280, 4), (33, 384, 2)])
def test_resid_layernorm_packed_vs_torch(M, D, nparts):
    x = torch.randn(M, D, device=DEV) * 3 + 1
    parts = torch.randn(max(nparts, 1), M, D, device=DEV)
    bias = torch.randn(D, device=DEV) if nparts else None
    g = torch.randn(D, device=DEV)
    b = torch.randn(D, device=DEV)
    out = torch.zeros(D * 64, dtype=torch.bfloat16, device=DEV)
    xr = x + (bias + parts[:nparts].sum(0) if nparts else 0)
    _lib.call("tw_resid_layernorm_packed", x.data_ptr(), parts.data_ptr(), nparts, _lib.ptr(bias), g.data_ptr(),
              b.data_ptr(), M, D, 1e-5, out.data_ptr(), S())
    torch.testing.assert_close(x, xr, atol=1e-5, rtol=1e-5)
    ref = torch.nn.functional.layer_norm(xr, (D,), g, b, 1e-5)
    torch.testing.assert_close(unpack_act(out, M, D).float(), ref, atol=3e-2, rtol=1e-2)
    # same bits as the row-major kernel
    rm = torch.empty(M, D, dtype=torch.bfloat16, device=DEV)
    x2 = torch.randn(M, D, device=DEV)
    x3 = x2.clone()
    _lib.call("tw_resid_layernorm", x2.data_ptr(), parts.data_ptr(), nparts, _lib.ptr(bias), g.data_ptr(), b.data_ptr(),
              M, D, 1e-5, rm.data_ptr(), S())
    _lib.call("tw_resid_layernorm_packed", x3.data_ptr(), parts.data_ptr(), nparts, _lib.ptr(bias), g.data_ptr(),
              b.data_ptr(), M, D, 1e-5, out.data_ptr(), S())
    assert torch.equal(unpack_act(out, M, D).view(torch.int16), rm.view(torch.int16))


def test_resid_layernorm_packed_to_writes_the_other_buffer():
    """tw_resid_layernorm_packed_to: the in-place kernel's arithmetic, the updated rows in x_out, x untouched."""
    M, D = 24, 1280
    x = torch.randn(M, D, device=DEV)
    parts = torch.randn(4, M, D, device=DEV)
    bias, g, b = torch.randn(D, device=DEV), torch.randn(D, device=DEV), torch.randn(D, device=DEV)
    x0 = x.clone()
    xo = torch.full_like(x, float("nan"))
    out1 = torch.zeros(D * 64, dtype=torch.bfloat16, device=DEV)
    out2 = torch.zeros_like(out1)
    _lib.call("tw_resid_layernorm_packed_to", x.data_ptr(), xo.data_ptr(), parts.data_ptr(), 4, bias.data_ptr(),
              g.data_ptr(), b.data_ptr(), M, D, 1e-5, out1.data_ptr(), S())
    x2 = x0.clone()
    _lib.call("tw_resid_layernorm_packed", x2.data_ptr(), parts.data_ptr(), 4, bias.data_ptr(), g.data_ptr(),
              b.data_ptr(), M, D, 1e-5, out2.data_ptr(), S())
    torch.cuda.synchronize()
    assert torch.equal(x, x0) and torch.equal(xo, x2) and torch.equal(out1, out2)

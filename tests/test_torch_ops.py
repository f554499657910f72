"""torch.ops.tw.* — the PyTorch-ROCm custom operators over the C-ABI (csrc/torch_ops.cpp).

CPU (no GPU needed): the operator library loads, every op of twamd._ops.OPS is registered with its schema, and the
Meta kernels give shapes (FakeTensor tracing of the encoder ops). GPU (`-m gpu`): the ops against the oracle /
torch fp32 exactly as the C-ABI kernel tests do (tolerances stated in each test), agreement with the C-ABI call
bit for bit, launch on torch's current stream, graph capture, and the engine's encoder routed through them."""
import numpy as np
import pytest
import torch

from oracle import whisper_oracle as wo
from twamd import _lib, _ops
from twamd.frontend import dft_basis, mel_table, pack_k8
from twamd.synth_audio import speech_like, white_noise


def test_ops_registered_with_schemas_and_meta_shapes():
    tw = _ops.load()
    for name in _ops.OPS:
        assert hasattr(tw, name), name
    assert "Tensor(a!) out" in str(tw.gemm_bf16_out.default._schema)
    meta = torch.device("meta")
    A = torch.empty(3000, 1280, dtype=torch.bfloat16, device=meta)
    W = torch.empty(3840, 1280, dtype=torch.bfloat16, device=meta)
    assert tw.gemm_bf16(A, W, _lib.TW_EPI_BF16).shape == (3000, 3840)
    assert tw.gemm_bf16(A, W, _lib.TW_EPI_F32).dtype == torch.float32
    qkv = torch.empty(3000, 3840, dtype=torch.bfloat16, device=meta)
    assert tw.attn_encoder(qkv, 2, 20).shape == (3000, 1280)
    wave = torch.empty(2, 480000, device=meta)
    assert tw.logmel(wave, wave, wave, wave, 128).shape == (2, 128, 3000)
    x = torch.empty(3000, 1280, device=meta)
    assert tw.layernorm(x, x[0], x[0], 1e-5).dtype == torch.bfloat16
    with pytest.raises(RuntimeError):  # the in-place epilogues have no functional form
        tw.gemm_bf16(A, W, _lib.TW_EPI_RESID_F32)


def test_fake_tensor_tracing_of_an_encoder_block():
    from torch._subclasses.fake_tensor import FakeTensorMode
    tw = _ops.load()
    with FakeTensorMode():
        x = torch.empty(3000, 1280)
        h = tw.layernorm(x, torch.empty(1280), torch.empty(1280), 1e-5)
        q = tw.gemm_bf16(h, torch.empty(3840, 1280, dtype=torch.bfloat16), _lib.TW_EPI_BF16, torch.empty(3840))
        a = tw.attn_encoder(q, 2, 20)
    assert a.shape == (3000, 1280) and a.dtype == torch.bfloat16


DEV = "cuda"


def _rand_bf16(*shape, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(torch.bfloat16).to(DEV)


@pytest.mark.gpu
def test_op_logmel_vs_oracle_and_capi():
    tw = _ops.load()
    clips = [speech_like(30.0, 1234), white_noise(12.3, 7)]
    wave = np.zeros((2, 480000), np.float32)
    for i, c in enumerate(clips):
        wave[i, : len(c)] = c[:480000]
    c, s = dft_basis()
    bc, bs, fb = (torch.from_numpy(pack_k8(a)).to(DEV) for a in (c, s, mel_table(128)))
    w = torch.from_numpy(wave).to(DEV)
    got = tw.logmel(w, bc, bs, fb, 128)
    feats = torch.empty_like(got)
    mk = torch.empty(2, dtype=torch.int32, device=DEV)
    _lib.call("tw_logmel", w.data_ptr(), 2, bc.data_ptr(), bs.data_ptr(), fb.data_ptr(), 128, feats.data_ptr(),
              mk.data_ptr(), torch.cuda.current_stream().cuda_stream)
    assert torch.equal(got, feats)  # the same kernel
    for i, cl in enumerate(clips):  # (the C-ABI kernel test's bound: f32 DFT-by-MFMA vs float64 FFT)
        np.testing.assert_allclose(got[i].cpu().numpy(), wo.log_mel(cl, 128), atol=1e-4, rtol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(1500, 1280, 1280), (300, 3840, 1280), (129, 200, 64)])
def test_op_gemm_bf16_vs_torch(M, N, K):
    tw = _ops.load()
    A = _rand_bf16(M, K, seed=1)
    W = _rand_bf16(N, K, scale=K ** -0.5, seed=2)
    bias = torch.randn(N, device=DEV) * 0.1
    ref = A.float() @ W.float().t() + bias
    out = tw.gemm_bf16(A, W, _lib.TW_EPI_BF16, bias)
    torch.testing.assert_close(out.float(), ref, atol=2e-2, rtol=2e-2)  # bf16 output
    f = tw.gemm_bf16(A, W, _lib.TW_EPI_F32, bias)
    torch.testing.assert_close(f, ref, atol=2e-3, rtol=2e-3)
    x = torch.randn(M, N, device=DEV)
    want = x + ref
    tw.gemm_bf16_out(A, W, _lib.TW_EPI_RESID_F32, x, bias)  # the residual update, in place
    torch.testing.assert_close(x, want, atol=2e-3, rtol=2e-3)


@pytest.mark.gpu
def test_op_attn_encoder_and_layernorm_vs_torch():
    tw = _ops.load()
    B, S, H = 2, 1500, 4
    qkv = _rand_bf16(B * S, 3 * H * 64, seed=5)
    D = H * 64
    qkv[:, :D] = (qkv[:, :D].float() * 0.125 * 3).to(torch.bfloat16)  # scaled q (as the C-ABI kernel test)
    out = tw.attn_encoder(qkv, B, H)
    capi = torch.empty_like(out)
    _lib.call("tw_attn_encoder", qkv.data_ptr(), B, S, H, capi.data_ptr(), torch.cuda.current_stream().cuda_stream)
    assert torch.equal(out.view(torch.int16), capi.view(torch.int16))  # the same kernel
    q, k, v = qkv.float().view(B, S, 3, H, 64).permute(2, 0, 3, 1, 4)
    ref = torch.softmax(q @ k.transpose(-1, -2), -1) @ v  # (q carries the 1/8 scale, as the packed weights do)
    torch.testing.assert_close(out.float().view(B, S, H, 64).permute(0, 2, 1, 3), ref, atol=2e-2, rtol=2e-2)
    x = torch.randn(3000, 1280, device=DEV) * 2 + 0.5
    g, b = torch.randn(1280, device=DEV), torch.randn(1280, device=DEV)
    got = tw.layernorm(x, g, b, 1e-5)
    torch.testing.assert_close(got.float(), torch.nn.functional.layer_norm(x, (1280,), g, b, 1e-5), atol=3e-2,
                               rtol=1e-2)


@pytest.mark.gpu
def test_ops_run_on_the_current_stream_and_capture():
    """An op launches on torch's current stream (ordered with torch work there) and records into a graph."""
    tw = _ops.load()
    A = _rand_bf16(600, 512, seed=3)
    W = _rand_bf16(384, 512, scale=512 ** -0.5, seed=4)
    out = torch.zeros(600, 384, dtype=torch.bfloat16, device=DEV)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            tw.gemm_bf16_out(A, W, _lib.TW_EPI_BF16, out)
    torch.cuda.current_stream().wait_stream(s)
    assert not out.float().abs().sum()  # captured, not run
    g.replay()
    torch.cuda.synchronize()
    torch.testing.assert_close(out.float(), A.float() @ W.float().t(), atol=2e-2, rtol=2e-2)
    with pytest.raises(RuntimeError, match="dtype"):
        tw.gemm_bf16(A.float(), W, _lib.TW_EPI_BF16)


@pytest.mark.gpu
def test_engine_encoder_runs_through_the_ops(monkeypatch):
    """The engine's encoder launches go through torch.ops.tw (counted), and its output equals the C-ABI path's."""
    from twamd.config import PRESETS, GenerationSettings
    from twamd.engine import WhisperEngine
    from twamd.weights import build_weights
    dims = PRESETS["test-mini"]
    eng = WhisperEngine(build_weights(dims, seed=1234), GenerationSettings.default(dims), max_batch=2, device="cuda")
    eng.wave[:2].copy_(torch.from_numpy(np.stack([speech_like(30.0, 1), speech_like(30.0, 2)])))
    calls = {}

    class Count:
        def __init__(self, ops):
            self._ops = ops

        def __getattr__(self, name):
            fn = getattr(self._ops, name)

            def wrapped(*a, **k):
                calls[name] = calls.get(name, 0) + 1
                return fn(*a, **k)
            return wrapped

    eng.ops = Count(eng.ops)
    eng.logmel(2)
    eng.row_map[:2] = torch.arange(2, dtype=torch.int32, device=DEV)
    eng.seek[:2] = 0
    eng.encode(2)
    torch.cuda.synchronize()
    L = dims.encoder_layers
    assert calls["logmel_out"] == 1 and calls["attn_encoder_out"] == L
    assert calls["gemm_bf16_out"] == 1 + 4 * L + 1  # conv1, q/k/v + o + fc1 + fc2 per layer, cross-K/V
    assert calls["layernorm_out"] == 2 * L + 1
    eng.close()


@pytest.mark.gpu
def test_ops_refuse_bad_operands():
    """a wrong-shaped call from Python is a TORCH_CHECK (RuntimeError naming the operand), never an
    out-of-bounds device access: cache / output / bias lengths, dtypes, the bf16 epilogue's 16-byte row stride."""
    tw = _ops.load()
    bf = torch.bfloat16
    B, H, T = 4, 2, 16
    qkv = torch.zeros(B, 3 * H * 64, dtype=bf, device=DEV)
    pos = torch.zeros(B, dtype=torch.int32, device=DEV)
    kc = torch.zeros(B * H * T * 64, dtype=bf, device=DEV)
    out = torch.zeros(B, H * 64, dtype=bf, device=DEV)
    tw.attn_decode_self_(qkv, H, T, pos, kc, kc.clone(), out)
    torch.cuda.synchronize()
    with pytest.raises(RuntimeError, match="k_cache"):
        tw.attn_decode_self_(qkv, H, T, pos, kc[:-64], kc.clone(), out)
    with pytest.raises(RuntimeError, match="pos"):
        tw.attn_decode_self_(qkv, H, T, pos.float(), kc, kc.clone(), out)
    with pytest.raises(RuntimeError, match="out"):
        tw.attn_decode_self_(qkv, H, T, pos, kc, kc.clone(), out[:2])
    cross = torch.zeros(2 * B * H * 100 * 64, dtype=bf, device=DEV)
    q = torch.zeros(B, H * 64, dtype=bf, device=DEV)
    tw.attn_decode_cross_out(q, H, 100, B, None, cross, out)
    with pytest.raises(RuntimeError, match="cross_kv"):
        tw.attn_decode_cross_out(q, H, 101, B, None, cross, out)
    A = torch.zeros(64, 64, dtype=bf, device=DEV)
    W = torch.zeros(128, 64, dtype=bf, device=DEV)
    with pytest.raises(RuntimeError, match="bias"):
        tw.gemm_bf16_out(A, W, _lib.TW_EPI_BF16, torch.empty(64, 128, dtype=bf, device=DEV),
                         torch.zeros(100, device=DEV))
    wide = torch.empty(64, 132, dtype=bf, device=DEV)[:, :128]  # row stride 132: not 16-byte aligned rows
    with pytest.raises(RuntimeError, match="multiple of 8"):
        tw.gemm_bf16_out(A, W, _lib.TW_EPI_BF16, wide)
    x = torch.zeros(24, 1280, device=DEV)
    g = torch.ones(1280, device=DEV)
    outp = torch.zeros(40 * 2 * 512, dtype=bf, device=DEV)
    tw.resid_layernorm_packed_(x, None, 0, None, g, g, 1e-5, outp)
    with pytest.raises(RuntimeError, match="gamma"):
        tw.resid_layernorm_packed_(x, None, 0, None, g[:1000], g, 1e-5, outp)
    with pytest.raises(RuntimeError, match="parts"):
        tw.resid_layernorm_packed_(x, torch.zeros(24 * 1280, device=DEV), 4, None, g, g, 1e-5, outp)
    torch.cuda.synchronize()

"""The oracle's MX fp8 restatement (config 5), pinned on CPU: e4m3 rounding and byte encoding against PyTorch's
own float8_e4m3fn conversion (round to nearest even, OCP e4m3fn), the scale rule's no-saturation property, and
the quantise-dequantise error bound of the format."""
import numpy as np
import torch

from oracle import whisper_oracle as wo


def test_e4m3_rounding_matches_torch_float8():
    rng = np.random.default_rng(0)
    y = (rng.uniform(-1, 1, 300000) * np.exp2(rng.integers(-16, 10, 300000))).astype(np.float32)
    y = np.clip(y, -448, 448)
    y[:6] = [0.0, -0.0, 448.0, -448.0, 1.0625, 1.1875]  # ties between e4m3 neighbours
    ours = wo.e4m3_rne(y)
    t = torch.from_numpy(y).to(torch.float8_e4m3fn)
    assert np.array_equal(ours, t.to(torch.float64).numpy())
    assert np.array_equal(wo.e4m3_bytes(ours), t.view(torch.uint8).numpy())


def test_mx_scale_rule_and_error_bound():
    rng = np.random.default_rng(1)
    x = (rng.standard_normal((64, 1280)) * np.exp2(rng.integers(-30, 20, (64, 1)))).astype(np.float32)
    x[0, :32] = 0.0
    x[1, :32] = 1.75 * 2.0 ** 3   # mantissa exactly 1.75: the lower scale still fits (448)
    x[2, :32] = 1.76 * 2.0 ** 3   # above 1.75: one scale step up
    q, s = wo.mx_quant(x)
    assert np.abs(q).max() <= 448.0
    assert s[0, 0] == 1 and np.all(q[0, :32] == 0)
    assert s[1, 0] == 127 + 3 - 8 and np.all(q[1, :32] == 448.0)
    assert s[2, 0] == 127 + 3 - 7
    xb = x.reshape(64, 40, 32)
    err = np.abs(wo.mx_dequant(q, s) - x).reshape(64, 40, 32)
    amax = np.abs(xb).max(-1, keepdims=True)
    # 3 mantissa bits: half a step of the block's top binade, which is <= amax / 8 (e4m3 normals inside the block)
    assert np.all(err <= amax / 16 + 1e-30 + np.ldexp(1.0, s[..., None].astype(np.int64) - 127 - 10))


def test_bf16_round_matches_torch():
    rng = np.random.default_rng(2)
    x = (rng.standard_normal(100000) * 10).astype(np.float32)
    assert np.array_equal(wo.bf16_round(x), torch.from_numpy(x).to(torch.bfloat16).float().numpy())


def test_encode_mx_close_to_fp32_encoder():
    """Config 5's reference encoder stays close to the fp32 one on a small seeded model (what MX fp8 costs)."""
    D, L, F, H = 128, 2, 512, 2
    sd = wo.synth_state_dict(D, L, 1, F, 80, 512, 7)
    m = wo.WhisperOracle(sd, H)
    rng = np.random.default_rng(3)
    feats = rng.uniform(-1, 1, (80, 3000)).astype(np.float32)
    a, b = m.encode(feats), m.encode_mx(feats)
    assert np.abs(a - b).mean() < 0.1
    assert np.abs(a - b).mean() > 1e-4  # it did quantise

"""CPU ORACLE (test infrastructure only) — numpy restatement of the reference's Whisper hot path.

NOT product code: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker. The product path (turbo-whisper-workspace_amd/twamd) never
imports it and has no CPU fallback.

What it restates (the reference executes transformers 5.15.0 here; it pins 4.54.1 / >=4.30.0,
see SURVEY.md §8c), float32 / float64 numpy:
  log-mel            WhisperFeatureExtractor._torch_extract_fbank_features
                     ($TF/models/whisper/feature_extraction_whisper.py:135-168), mel_filter_bank
                     ($TF/audio_utils.py:638-729)
  encoder            WhisperEncoder.forward ($TF/models/whisper/modeling_whisper.py:592-646),
                     WhisperEncoderLayer (:360-413), WhisperAttention (:241-356)
  decoder step       WhisperDecoder.forward / WhisperDecoderLayer (:690-795, 416-505), tied proj_out
  processors         SuppressTokensAtBegin / SuppressTokens / WhisperTimeStamp
                     ($TF/generation/logits_process.py:1816-2047)
  greedy loop        GenerationMixin._sample ($TF/generation/utils.py:2783-2941)
  seek loop          WhisperGenerationMixin.generate / generate_with_fallback / _retrieve_segment
                     ($TF/models/whisper/generation_whisper.py:785-903, 970-1116, 1977-2074)
  synthetic weights  tw_fill_synth (turbo-whisper-workspace_amd/csrc/tw_runtime.hip)

Pinning: tests/test_oracle_golden.py checks every function above against golden vectors that
tests/golden/make_golden.py produced by running transformers itself on the same seeded weights.
"""
from __future__ import annotations

import math
import zlib
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

# ----------------------------------------------------------------------------- synthetic parameters
_M64 = (1 << 64) - 1


def synth_uniform(seed: int, tensor_id: int, n: int, scale: float, offset: float) -> np.ndarray:
    """Bit-exact numpy restatement of k_fill_synth: bf16-rounded uniform(-1,1)*scale+offset, as f32."""
    idx = np.arange(n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z0 = (np.uint64((seed * 0x9E3779B97F4A7C15) & _M64)
              ^ np.uint64(((tensor_id + 1) * 0xD1B54A32D192ED03) & _M64))
        z = z0 + idx * np.uint64(0x9E3779B97F4A7C15)
        z ^= z >> np.uint64(30)
        z *= np.uint64(0xBF58476D1CE4E5B9)
        z ^= z >> np.uint64(27)
        z *= np.uint64(0x94D049BB133111EB)
        z ^= z >> np.uint64(31)
    s = (z >> np.uint64(40)).astype(np.int64) - 8388608
    u = (2 * s + 1).astype(np.float32) * np.float32(1.0 / 16777216.0)
    v = (u * np.float32(scale)).astype(np.float32) + np.float32(offset)
    v = v.astype(np.float32)
    bits = v.view(np.uint32).astype(np.uint64)
    rnd = (bits + np.uint64(0x7FFF) + ((bits >> np.uint64(16)) & np.uint64(1))) >> np.uint64(16)
    return (rnd.astype(np.uint32) << np.uint32(16)).view(np.float32)


def param_shapes(D: int, L_enc: int, L_dec: int, F: int, n_mels: int, V: int,
                 n_src: int = 1500, n_tgt: int = 448) -> List[Tuple[str, Tuple[int, ...]]]:
    out = [("model.encoder.conv1.weight", (D, n_mels, 3)), ("model.encoder.conv1.bias", (D,)),
           ("model.encoder.conv2.weight", (D, D, 3)), ("model.encoder.conv2.bias", (D,)),
           ("model.encoder.embed_positions.weight", (n_src, D))]

    def attn(p):
        out.extend([(f"{p}.k_proj.weight", (D, D)), (f"{p}.v_proj.weight", (D, D)), (f"{p}.v_proj.bias", (D,)),
                    (f"{p}.q_proj.weight", (D, D)), (f"{p}.q_proj.bias", (D,)),
                    (f"{p}.out_proj.weight", (D, D)), (f"{p}.out_proj.bias", (D,))])

    def ln(p):
        out.extend([(f"{p}.weight", (D,)), (f"{p}.bias", (D,))])

    def mlp(p):
        out.extend([(f"{p}.fc1.weight", (F, D)), (f"{p}.fc1.bias", (F,)),
                    (f"{p}.fc2.weight", (D, F)), (f"{p}.fc2.bias", (D,))])

    for i in range(L_enc):
        p = f"model.encoder.layers.{i}"
        attn(f"{p}.self_attn"); ln(f"{p}.self_attn_layer_norm"); mlp(p); ln(f"{p}.final_layer_norm")
    ln("model.encoder.layer_norm")
    out += [("model.decoder.embed_tokens.weight", (V, D)), ("model.decoder.embed_positions.weight", (n_tgt, D))]
    for i in range(L_dec):
        p = f"model.decoder.layers.{i}"
        attn(f"{p}.self_attn"); ln(f"{p}.self_attn_layer_norm")
        attn(f"{p}.encoder_attn"); ln(f"{p}.encoder_attn_layer_norm")
        mlp(p); ln(f"{p}.final_layer_norm")
    ln("model.decoder.layer_norm")
    return out


def synth_spec(name: str, shape: Tuple[int, ...], D: int) -> Tuple[int, float, float]:
    tid = zlib.crc32(name.encode()) & 0xFFFFFFFF
    if "layer_norm" in name:
        return (tid, 0.2, 1.0) if name.endswith("weight") else (tid, 0.1, 0.0)
    if name.endswith("embed_tokens.weight"):
        return tid, (3.0 ** 0.5) * 2.0 / (D ** 0.5), 0.0
    if name.endswith("embed_positions.weight"):
        return tid, 0.5, 0.0
    if name.endswith("bias"):
        return tid, 0.05, 0.0
    fan_in = int(np.prod(shape[1:]))
    return tid, (3.0 / fan_in) ** 0.5, 0.0


def synth_state_dict(D, L_enc, L_dec, F, n_mels, V, seed) -> Dict[str, np.ndarray]:
    """Every parameter, generated tensor by tensor on a thread pool (numpy's integer ufuncs release the GIL)."""
    import concurrent.futures
    import os

    shapes = param_shapes(D, L_enc, L_dec, F, n_mels, V)

    def one(item):
        name, shape = item
        tid, scale, off = synth_spec(name, shape, D)
        return name, synth_uniform(seed, tid, int(np.prod(shape)), scale, off).reshape(shape)

    with concurrent.futures.ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 1)) as ex:
        return dict(ex.map(one, shapes))


# ----------------------------------------------------------------------------- log-mel
def _hz_to_mel(f):
    f = np.asarray(f, np.float64)
    return np.where(f >= 1000.0, 15.0 + np.log(np.maximum(f, 1e-300) / 1000.0) * (27.0 / np.log(6.4)), 3.0 * f / 200.0)


def _mel_to_hz(m):
    m = np.asarray(m, np.float64)
    return np.where(m >= 15.0, 1000.0 * np.exp(np.log(6.4) / 27.0 * (m - 15.0)), 200.0 * m / 3.0)


def mel_filters(n_mels: int) -> np.ndarray:
    pts = _mel_to_hz(np.linspace(_hz_to_mel(0.0), _hz_to_mel(8000.0), n_mels + 2))
    fft = np.linspace(0, 8000, 201)
    diff = np.diff(pts)
    slopes = pts[None, :] - fft[:, None]
    fb = np.maximum(0.0, np.minimum(-slopes[:, :-2] / diff[:-1], slopes[:, 2:] / diff[1:]))
    return fb * (2.0 / (pts[2: n_mels + 2] - pts[:n_mels]))[None, :]


def log_mel(wave: np.ndarray, n_mels: int, long: bool = False) -> np.ndarray:
    """One 30-s window (padded/truncated to 480000) -> f32 [n_mels][3000]. long: the whole input as it is (the
    feature extractor with truncation=False, padding="longest" on one sequence, asr:450-457) -> [n_mels][n // 160],
    the max - 8 clamp over all of it (feature_extraction_whisper.py:135-168)."""
    if long:
        x = np.asarray(wave, np.float32).astype(np.float64)
    else:
        x = np.zeros(480000, np.float64)
        w = np.asarray(wave, np.float32)[:480000]
        x[: len(w)] = w
    nfr = len(x) // 160
    xp = np.pad(x, (200, 200), mode="reflect")
    idx = np.arange(nfr + 1)[:, None] * 160 + np.arange(400)[None, :]
    n = np.arange(400)
    win = 0.5 - 0.5 * np.cos(2 * np.pi * n / 400)
    spec = np.fft.rfft(xp[idx] * win[None, :], axis=1)          # [3001][201]
    mag = (np.abs(spec[:-1]) ** 2).T                               # [201][frames]
    mel = mel_filters(n_mels).T.astype(np.float32).astype(np.float64) @ mag
    ls = np.log10(np.maximum(mel, 1e-10))
    ls = np.maximum(ls, ls.max() - 8.0)
    return ((ls + 4.0) / 4.0).astype(np.float32)


# ----------------------------------------------------------------------------- model
def _gelu(x):
    from scipy.special import erf

    return 0.5 * x * (1.0 + erf(x / np.sqrt(2.0)))


def _ln(x, g, b, eps=1e-5):
    m = x.mean(-1, keepdims=True)
    v = ((x - m) ** 2).mean(-1, keepdims=True)
    return (x - m) / np.sqrt(v + eps) * g + b


def _softmax(x):
    x = x - x.max(-1, keepdims=True)
    e = np.exp(x)
    return e / e.sum(-1, keepdims=True)


# ----------------------------------------------------------------------------- MX fp8 (BASELINE config 5)
# Not in the reference: config 5 ("fp8 MFMA encoder + bf16 decoder") runs the encoder projections of
# modeling_whisper.py:279-282,309,375-376 on OCP MX fp8 operands. This restates the format the kernels use
# (turbo-whisper-workspace_amd/csrc/tw_common.h "MX fp8"): e4m3fn elements, one e8m0 scale per 32 K elements,
# s = E(absmax) - 8 (+1 when the absmax mantissa exceeds 1.75, so nothing saturates; 1 for E < 9),
# element = rne_e4m3(clip(x * 2^(127-s), +-448)).

def e4m3_rne(y: np.ndarray) -> np.ndarray:
    """Round |y| <= 448 to the nearest OCP e4m3fn value (ties to even), as float64."""
    y = np.asarray(y, np.float64)
    _, ex = np.frexp(y)                      # y = m * 2^ex, m in [0.5, 1): floor(log2|y|) = ex - 1
    e = np.maximum(ex - 1, -6)               # subnormals share the exponent -6
    step = np.ldexp(1.0, e - 3)              # 3 mantissa bits
    return np.round(y / step) * step         # np.round: half to even


def mx_quant(x: np.ndarray):
    """x [..., K] (K % 32 == 0) -> (elements e4m3 as float64 [..., K], scale bytes uint8 [..., K/32])."""
    x = np.asarray(x, np.float32)
    xb = x.reshape(x.shape[:-1] + (x.shape[-1] // 32, 32))
    amax = np.abs(xb).max(-1).astype(np.float32)
    u = amax.view(np.uint32).astype(np.int64)
    E = (u >> 23) & 0xFF
    s = np.where(E < 9, 1, E - 8 + ((u & 0x7FFFFF) > 0x600000)).astype(np.uint8)
    inv = np.ldexp(1.0, 127 - s.astype(np.int64))[..., None]
    q = e4m3_rne(np.clip(xb.astype(np.float64) * inv, -448.0, 448.0))
    return q.reshape(x.shape), s


def mx_dequant(q: np.ndarray, s: np.ndarray) -> np.ndarray:
    qb = q.reshape(q.shape[:-1] + (q.shape[-1] // 32, 32))
    return (qb * np.ldexp(1.0, s.astype(np.int64) - 127)[..., None]).reshape(q.shape)


def mx_round(x: np.ndarray) -> np.ndarray:
    """Quantise-dequantise: the value an MX fp8 GEMM operand carries, float32."""
    return mx_dequant(*mx_quant(x)).astype(np.float32)


def e4m3_bytes(q: np.ndarray) -> np.ndarray:
    """e4m3fn encoding (uint8) of exactly representable float64 values (|q| <= 448)."""
    q = np.asarray(q, np.float64)
    sign = (q < 0) | ((q == 0) & np.signbit(q))
    a = np.abs(q)
    _, ex = np.frexp(a)
    e = np.maximum(ex - 1, -6)
    mant = np.round(a / np.ldexp(1.0, e - 3)).astype(np.int64)  # 8..15 normal, 0..7 subnormal
    normal = mant >= 8
    code = np.where(normal, ((e + 7) << 3) | (mant - 8), mant)
    return (code | (sign.astype(np.int64) << 7)).astype(np.uint8)


def bf16_round(x: np.ndarray) -> np.ndarray:
    """float32 -> nearest bf16 (ties to even), returned as float32."""
    u = np.asarray(x, np.float32).view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000
    return u.astype(np.uint32).view(np.float32)


class WhisperOracle:
    """fp32 numpy Whisper with the HF parameter names."""

    def __init__(self, sd: Dict[str, np.ndarray], heads: int):
        self.sd = {k: np.asarray(v, np.float32) for k, v in sd.items()}
        self.H = heads
        self.D = self.sd["model.encoder.conv1.bias"].shape[0]
        self.L_enc = sum(1 for k in sd if k.startswith("model.encoder.layers.") and k.endswith("fc1.bias"))
        self.L_dec = sum(1 for k in sd if k.startswith("model.decoder.layers.") and k.endswith("fc1.bias"))

    def _lin(self, x, p, bias=True):
        y = x @ self.sd[f"{p}.weight"].T
        if bias and f"{p}.bias" in self.sd:
            y = y + self.sd[f"{p}.bias"]
        return y

    def _mha(self, xq, xkv, p, k=None, v=None, probs_out=None):
        """Multi-head attention; q scaled by head_dim^-0.5 before QK^T (modeling_whisper.py:309).
        probs_out: list that receives the attention probabilities [H][T][S]."""
        H, hd = self.H, self.D // self.H
        q = self._lin(xq, f"{p}.q_proj") * (hd ** -0.5)
        if k is None:
            k = self._lin(xkv, f"{p}.k_proj", bias=False)
            v = self._lin(xkv, f"{p}.v_proj")
        T, S = q.shape[0], k.shape[0]
        qh = q.reshape(T, H, hd).transpose(1, 0, 2)
        kh = k.reshape(S, H, hd).transpose(1, 0, 2)
        vh = v.reshape(S, H, hd).transpose(1, 0, 2)
        pr = _softmax(qh @ kh.transpose(0, 2, 1))
        if probs_out is not None:
            probs_out.append(pr)
        o = pr @ vh
        return self._lin(o.transpose(1, 0, 2).reshape(T, self.D), f"{p}.out_proj")

    def conv_stem(self, feats: np.ndarray) -> np.ndarray:
        """feats [n_mels][3000] -> x [1500][D] (gelu(conv1) -> gelu(conv2) -> + positions)."""
        sd = self.sd

        def conv(x, w, b, stride):
            C, T = x.shape
            xp = np.pad(x, ((0, 0), (1, 1)))
            To = (T + 2 - 3) // stride + 1
            cols = np.stack([xp[:, j: j + stride * (To - 1) + 1: stride] for j in range(3)], 0)  # [3][C][To]
            return np.einsum("ocj,jct->ot", w, cols, optimize=True) + b[:, None]

        h = _gelu(conv(feats.astype(np.float32), sd["model.encoder.conv1.weight"], sd["model.encoder.conv1.bias"], 1))
        h = _gelu(conv(h.astype(np.float32), sd["model.encoder.conv2.weight"], sd["model.encoder.conv2.bias"], 2))
        return (h.T + sd["model.encoder.embed_positions.weight"]).astype(np.float32)

    def encode(self, feats: np.ndarray) -> np.ndarray:
        x = self.conv_stem(feats)
        for i in range(self.L_enc):
            p = f"model.encoder.layers.{i}"
            sd = self.sd
            h = _ln(x, sd[f"{p}.self_attn_layer_norm.weight"], sd[f"{p}.self_attn_layer_norm.bias"])
            x = x + self._mha(h, h, f"{p}.self_attn")
            h = _ln(x, sd[f"{p}.final_layer_norm.weight"], sd[f"{p}.final_layer_norm.bias"])
            x = x + self._lin(_gelu(self._lin(h, f"{p}.fc1")), f"{p}.fc2")
            x = x.astype(np.float32)
        return _ln(x, self.sd["model.encoder.layer_norm.weight"], self.sd["model.encoder.layer_norm.bias"]).astype(np.float32)

    def _lin_mx(self, xq, p, scale=1.0):
        """nn.Linear on MX operands: mx_round(x) . mx_round(scale * W)^T + scale * b (scale: the 2^-3 folded into
        the packed q rows, exact in MX)."""
        w = mx_round(self.sd[f"{p}.weight"] * np.float32(scale))
        y = xq.astype(np.float64) @ w.T.astype(np.float64)
        if f"{p}.bias" in self.sd:
            y = y + self.sd[f"{p}.bias"] * np.float32(scale)
        return y.astype(np.float32)

    def encode_mx(self, feats: np.ndarray) -> np.ndarray:
        """The config-5 encoder: conv stem, attention core and LayerNorms as encode(); the q/k/v/o and fc1/fc2
        projections on MX fp8 operands quantised where the GPU quantises them (LayerNorm output, attention output
        and GELU(fc1), each from f32)."""
        sd, H, hd = self.sd, self.H, self.D // self.H
        x = self.conv_stem(feats)
        for i in range(self.L_enc):
            p = f"model.encoder.layers.{i}"
            h = mx_round(_ln(x, sd[f"{p}.self_attn_layer_norm.weight"], sd[f"{p}.self_attn_layer_norm.bias"]))
            q = self._lin_mx(h, f"{p}.self_attn.q_proj", hd ** -0.5)
            k = self._lin_mx(h, f"{p}.self_attn.k_proj")
            v = self._lin_mx(h, f"{p}.self_attn.v_proj")
            T = q.shape[0]
            qh, kh, vh = (t.reshape(T, H, hd).transpose(1, 0, 2) for t in (q, k, v))
            o = (_softmax(qh @ kh.transpose(0, 2, 1)) @ vh).transpose(1, 0, 2).reshape(T, self.D)
            x = x + self._lin_mx(mx_round(o), f"{p}.self_attn.out_proj")
            h = mx_round(_ln(x, sd[f"{p}.final_layer_norm.weight"], sd[f"{p}.final_layer_norm.bias"]))
            x = (x + self._lin_mx(mx_round(_gelu(self._lin_mx(h, f"{p}.fc1"))), f"{p}.fc2")).astype(np.float32)
        return _ln(x, sd["model.encoder.layer_norm.weight"], sd["model.encoder.layer_norm.bias"]).astype(np.float32)

    def new_cache(self, enc: np.ndarray, pos0: int = 0) -> dict:
        """pos0: the position of the first token fed — a row left padded by pos0 tokens that its queries never attend
        (generate()'s decoder_attention_mask over a conditioned batch) computes exactly this: pads take positions,
        nothing else."""
        cross = []
        for i in range(self.L_dec):
            p = f"model.decoder.layers.{i}.encoder_attn"
            cross.append((self._lin(enc, f"{p}.k_proj", bias=False), self._lin(enc, f"{p}.v_proj")))
        return {"self": [(np.zeros((0, self.D), np.float32), np.zeros((0, self.D), np.float32))
                         for _ in range(self.L_dec)], "cross": cross, "len": pos0}

    def decoder_step(self, token: int, cache: dict) -> np.ndarray:
        """One token at position cache['len'] -> f32 logits [V] (updates cache)."""
        sd, t = self.sd, cache["len"]
        x = (sd["model.decoder.embed_tokens.weight"][token] + sd["model.decoder.embed_positions.weight"][t])[None, :]
        for i in range(self.L_dec):
            p = f"model.decoder.layers.{i}"
            h = _ln(x, sd[f"{p}.self_attn_layer_norm.weight"], sd[f"{p}.self_attn_layer_norm.bias"])
            kk, vv = cache["self"][i]
            kk = np.concatenate([kk, self._lin(h, f"{p}.self_attn.k_proj", bias=False)], 0)
            vv = np.concatenate([vv, self._lin(h, f"{p}.self_attn.v_proj")], 0)
            cache["self"][i] = (kk, vv)
            x = x + self._mha(h, None, f"{p}.self_attn", kk, vv)
            h = _ln(x, sd[f"{p}.encoder_attn_layer_norm.weight"], sd[f"{p}.encoder_attn_layer_norm.bias"])
            ck, cv = cache["cross"][i]
            rec = [] if "xattn" in cache else None
            x = x + self._mha(h, None, f"{p}.encoder_attn", ck, cv, probs_out=rec)
            if rec is not None:  # cross-attention probabilities of this step, [H][S], per layer
                cache["xattn"].setdefault(t, {})[i] = rec[0][:, 0, :]
            h = _ln(x, sd[f"{p}.final_layer_norm.weight"], sd[f"{p}.final_layer_norm.bias"])
            x = x + self._lin(_gelu(self._lin(h, f"{p}.fc1")), f"{p}.fc2")
        cache["len"] = t + 1
        h = _ln(x, sd["model.decoder.layer_norm.weight"], sd["model.decoder.layer_norm.bias"])
        return (sd["model.decoder.embed_tokens.weight"] @ h[0]).astype(np.float32)  # tied proj_out (row-major GEMV)


# ----------------------------------------------------------------------------- generation
class GenCfg:
    """The generation fields the Whisper greedy path reads (plain ints, no product imports)."""

    def __init__(self, V, eot, sot, lang_begin, n_lang, transcribe, translate, notimestamps, suppress_tokens,
                 begin_suppress_tokens, max_initial_timestamp_index=50, max_length=448, multilingual=True):
        self.V, self.eot, self.sot = V, eot, sot
        self.lang_begin, self.n_lang = lang_begin, n_lang
        self.transcribe, self.translate, self.notimestamps = transcribe, translate, notimestamps
        self.ts_begin = notimestamps + 1
        self.suppress = list(suppress_tokens)
        self.begin_suppress = list(begin_suppress_tokens)
        self.mit = max_initial_timestamp_index
        self.max_length = max_length
        self.multilingual = multilingual


def process_logits(scores: np.ndarray, sampled: Sequence[int], g: GenCfg, use_ts: bool) -> np.ndarray:
    """The processor chain of _retrieve_logit_processors applied to one row (f32)."""
    if not use_ts:
        s = scores.astype(np.float32).copy()
        if len(sampled) == 0 and g.begin_suppress:
            s[g.begin_suppress] = -np.inf
        if g.suppress:
            s[g.suppress] = -np.inf
        return s
    s = process_logits_no_rule(scores, sampled, g)
    margin = _ts_rule_margin(s, g.ts_begin)
    if margin > 0:  # "if sum of probability over timestamps is above any other token, sample timestamp"
        s[: g.ts_begin] = -np.inf
    return s


def _ts_rule_margin(s: np.ndarray, tb: int) -> float:
    """logsumexp(timestamp log-probs) - max(text log-probs) of processed scores s (WhisperTimeStampLogits-
    Processor, logits_process.py:2041-2045); > 0 forces a timestamp."""
    with np.errstate(divide="ignore", invalid="ignore"):
        m = np.max(s)
        if not np.isfinite(m):
            return -np.inf
        lp = s - (m + np.log(np.sum(np.exp(s - m))))
        ts_lp = lp[tb:]
        mt = np.max(ts_lp)
        ts_lse = mt + np.log(np.sum(np.exp(ts_lp - mt))) if np.isfinite(mt) else -np.inf
        return float(ts_lse - np.max(lp[:tb]))


def greedy_pass(model: WhisperOracle, enc: np.ndarray, prompt: Sequence[int], max_new: int, g: GenCfg,
                use_ts: bool, logits_out: Optional[list] = None, xattn: Optional[dict] = None,
                cache_out: Optional[list] = None) -> List[int]:
    """_sample for one row: returns the generated tokens (incl. the EOS), or up to max_new.
    xattn: dict that receives the cross-attention probabilities of every fed position ({pos: {layer: [H][S]}}).
    cache_out: receives the row's KV cache (a batch keeps feeding pad tokens to finished rows)."""
    cache = model.new_cache(enc)
    if cache_out is not None:
        cache_out.append(cache)
    if xattn is not None:
        cache["xattn"] = xattn
    for t in prompt[:-1]:
        model.decoder_step(t, cache)
    logits = model.decoder_step(prompt[-1], cache)
    out: List[int] = []
    while True:
        s = process_logits(logits, out, g, use_ts)
        if logits_out is not None:
            logits_out.append((logits.copy(), s))
        tok = int(np.argmax(s))
        out.append(tok)
        if tok == g.eot or len(out) >= max_new:
            return out
        logits = model.decoder_step(tok, cache)


def _log_softmax32(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.float32)
    m = np.max(x)
    return (x - (m + np.log(np.sum(np.exp(x - m), dtype=np.float32)))).astype(np.float32)


def _topk_desc(x: np.ndarray, k: int) -> np.ndarray:
    """Indices of the k largest values, descending; ties -> lower index first."""
    if x.size <= 4 * k:
        return np.argsort(-x, kind="stable")[:k]
    kth = np.partition(x, x.size - k)[x.size - k]
    cand = np.nonzero(x >= kth)[0]  # every value tied with the k-th is a candidate
    return cand[np.lexsort((cand, -x[cand]))][:k]


def beam_search_core(first_logits: np.ndarray, step_fn, P: int, max_new: int, g: GenCfg, use_ts: bool,
                     num_beams: int, length_penalty: float = 1.0) -> Tuple[List[int], dict]:
    """GenerationMixin._beam_search ($TF/generation/utils.py:3208-3512) for ONE window with the Whisper processor
    chain, early_stopping=False (GenerationConfig default), one EOS id: K = 2 * num_beams continuations per step
    (:3277-3282) from log_softmax(f32 logits) + processors (:3381-3382) + the running beam scores; running beams =
    best K non-finished (:3131-3151); finished beams = best of the previous and the just-finished top-num_beams
    candidates scored sum/len**length_penalty (:3153-3206); stop when no running beam can beat the worst finished
    one (:3008-3053) or every candidate hit a stopping criterion (EOS / max_length, :3055-3073).
    first_logits: f32[V] after the prompt; step_fn(src_beams, tokens) -> f32[nb][V]: reorder the beams' decoder
    caches to src_beams, feed tokens, return the next logits. Returns (generated tokens of the best finished beam,
    with its EOS if it ended on one; a trace dict of the final finished/running beams)."""
    nb, K, V = num_beams, 2 * num_beams, g.V
    max_length = P + max_new
    logits = [first_logits] * nb
    run_tok: List[List[int]] = [[] for _ in range(nb)]
    run_score = np.full(nb, -1e9, np.float32)
    run_score[0] = 0.0
    fin_score = np.full(nb, -1e9, np.float32)
    fin_seq: List[List[int]] = [[] for _ in range(nb)]
    fin_flag = np.zeros(nb, bool)
    unsatisfied = True
    cur_len = P
    while True:
        acc = np.empty(nb * V, np.float32)
        for b in range(nb):
            lp = process_logits(_log_softmax32(logits[b]), run_tok[b], g, use_ts)
            acc[b * V:(b + 1) * V] = lp + run_score[b]
        top = _topk_desc(acc, K)
        sc = acc[top].astype(np.float32)
        src, tok = top // V, top % V
        hits = (tok == g.eot) | (cur_len + 1 >= max_length)
        # e. running beams for the next step
        rsc = (sc + hits.astype(np.float32) * np.float32(-1e9)).astype(np.float32)
        order = _topk_desc(rsc, nb)
        # f. finished beams
        cand = (sc / np.float32((cur_len + 1 - P) ** length_penalty)).astype(np.float32)
        if not unsatisfied:
            cand = cand + np.float32(-1e9)
        just = hits & (np.arange(K) < nb)
        cand = np.where(just, cand, cand + np.float32(-1e9)).astype(np.float32)
        merged = np.concatenate([fin_score, cand])
        msel = _topk_desc(merged, nb)
        new_seq, new_flag = [], []
        for i in msel:
            if i < nb:
                new_seq.append(fin_seq[i])
                new_flag.append(fin_flag[i])
            else:
                c = i - nb
                new_seq.append(run_tok[src[c]] + [int(tok[c])])
                new_flag.append(bool(just[c]))
        fin_score, fin_seq, fin_flag = merged[msel].astype(np.float32), new_seq, np.array(new_flag)
        # g. reorder the running beams
        srcs = [int(src[c]) for c in order]
        run_tok = [run_tok[src[c]] + [int(tok[c])] for c in order]
        run_score = rsc[order].astype(np.float32)
        cur_len += 1
        best_possible = run_score[0] / np.float32((cur_len - P) ** length_penalty)
        worst = np.where(fin_flag, np.min(fin_score), np.float32(-1e9))
        unsatisfied = unsatisfied and bool(np.any(best_possible > worst))
        if not unsatisfied or bool(np.all(hits)):
            break
        logits = step_fn(srcs, [t[-1] for t in run_tok])
    trace = {"fin_score": fin_score, "fin_seq": fin_seq, "fin_flag": fin_flag, "run_tok": run_tok,
             "run_score": run_score, "steps": cur_len - P}
    return list(fin_seq[0]), trace


def beam_pass(model: WhisperOracle, enc: np.ndarray, prompt: Sequence[int], max_new: int, g: GenCfg, use_ts: bool,
              num_beams: int, length_penalty: float = 1.0) -> List[int]:
    """beam_search_core driven by the oracle decoder (one KV cache per beam, reordered like the model's cache)."""
    base = model.new_cache(enc)
    for t in prompt[:-1]:
        model.decoder_step(t, base)
    logits0 = model.decoder_step(prompt[-1], base)

    def clone(c):
        return {"self": [(k.copy(), v.copy()) for k, v in c["self"]], "cross": c["cross"], "len": c["len"]}

    caches = [clone(base) for _ in range(num_beams)]

    def step(srcs, toks):
        new = [clone(caches[s]) for s in srcs]
        caches[:] = new
        return [model.decoder_step(t, c) for t, c in zip(toks, caches)]

    return beam_search_core(logits0, step, len(prompt), max_new, g, use_ts, num_beams, length_penalty)[0]


# ----------------------------------------------------------------------------- token-level timestamps
def median_filter(x: np.ndarray, width: int) -> np.ndarray:
    """_median_filter ($TF/models/whisper/generation_whisper.py:43-61): reflect-pad the last axis by width//2, the
    middle of the sorted window (NaN sorts last, as torch.sort)."""
    pad = width // 2
    if x.shape[-1] <= pad:
        return x
    xp = np.pad(x, [(0, 0)] * (x.ndim - 1) + [(pad, pad)], mode="reflect")
    win = np.lib.stride_tricks.sliding_window_view(xp, width, axis=-1)
    return np.sort(win, axis=-1)[..., pad]


def dynamic_time_warping(matrix: np.ndarray):
    """_dynamic_time_warping (generation_whisper.py:64-114), restated: float32 cost table, ties resolved to the
    horizontal move, backtrace from the corner. Returns (text_indices, time_indices)."""
    n, m = matrix.shape
    cost = np.full((n + 1, m + 1), np.inf, np.float32)
    trace = -np.ones((n + 1, m + 1), np.float32)
    cost[0, 0] = 0
    for j in range(1, m + 1):
        for i in range(1, n + 1):
            c0, c1, c2 = cost[i - 1, j - 1], cost[i - 1, j], cost[i, j - 1]
            if c0 < c1 and c0 < c2:
                c, t = c0, 0
            elif c1 < c0 and c1 < c2:
                c, t = c1, 1
            else:
                c, t = c2, 2
            cost[i, j] = matrix[i - 1, j - 1] + c
            trace[i, j] = t
    i, j = n, m
    trace[0, :] = 2
    trace[:, 0] = 1
    ti, tj = [], []
    while i > 0 or j > 0:
        ti.append(i - 1)
        tj.append(j - 1)
        if trace[i, j] == 0:
            i -= 1
            j -= 1
        elif trace[i, j] == 1:
            i -= 1
        else:
            j -= 1
    return np.array(ti[::-1]), np.array(tj[::-1])


def token_timestamps(weights: np.ndarray, num_input_ids: int, num_frames: Optional[int], median_width: int = 7,
                     time_precision: float = 0.02) -> np.ndarray:
    """_extract_token_timestamps (generation_whisper.py:241-380) for ONE sequence, num_beams=1.
    weights: f32 [heads][rows][1500], the alignment heads' cross-attention of every fed token (prompt rows first);
    returns f32 timestamps of length rows + 1."""
    heads, rows, _ = weights.shape
    ts = np.zeros(rows + 1, np.float32)
    w = weights.astype(np.float32)
    if num_frames is not None:
        # generate() passes num_frames as a per-sample tensor (attention_mask.sum - seek): the weights are cropped
        # once for the batch (:316-323) and once more per sample (:353-354); only a negative value (a seek past the
        # audio end, e.g. -390 // 2) makes the second crop bite
        w = w[..., : num_frames // 2]
        w = w[..., : num_frames // 2]
    w = w[:, num_input_ids:, :]
    if w.shape[1] == 0:
        return ts
    with np.errstate(invalid="ignore", divide="ignore"):
        std = w.std(axis=-2, keepdims=True)
        mean = w.mean(axis=-2, keepdims=True)
        w = ((w - mean) / std).astype(np.float32)
    w = median_filter(w, median_width)
    mat = w.mean(axis=0)
    text_idx, time_idx = dynamic_time_warping(-mat.astype(np.float64))
    jumps = np.pad(np.diff(text_idx), (1, 0), constant_values=1).astype(bool)
    jump_times = time_idx[jumps] * time_precision
    return np.concatenate([np.zeros(num_input_ids), jump_times, [jump_times[-1]]]).astype(np.float32)


def detect_language(model: WhisperOracle, enc: np.ndarray, g: GenCfg) -> int:
    cache = model.new_cache(enc)
    lg = model.decoder_step(g.sot, cache)
    m = np.full_like(lg, -np.inf)
    m[g.lang_begin: g.lang_begin + g.n_lang] = lg[g.lang_begin: g.lang_begin + g.n_lang]
    return int(np.argmax(m))


def segment_input(feats: np.ndarray, seek: int, max_frames: int = 3000) -> np.ndarray:
    """_get_input_segment (generation_whisper.py:1831-1850): feats[:, seek : seek + seek_num_frames], seek_num_frames =
    min(max_frames - seek, 3000), zero padded to 3000 frames."""
    snf = min(max_frames - seek, 3000)
    seg = np.zeros((feats.shape[0], 3000), np.float32)
    seg[:, :snf] = feats[:, seek: seek + snf]
    return seg


def retrieve_segment(seq, seek_num_frames, tb):
    ts = [t >= tb for t in seq]
    single = ts[-2:] == [False, True]
    pairs = [i + 1 for i in range(len(seq) - 1) if ts[i] and ts[i + 1]]
    if pairs:
        if single:
            return list(seq), seek_num_frames
        end = pairs[-1] + 1
        return list(seq[:end]), (seq[end - 2] - tb) * 2
    return list(seq), seek_num_frames


def generate(model: WhisperOracle, feats: np.ndarray, g: GenCfg, task: Optional[str] = "transcribe",
             language: Optional[int] = None, return_timestamps: bool = True, max_new_tokens: Optional[int] = None,
             encoder_cache: Optional[dict] = None, num_beams: int = 1, alignment_heads=None,
             num_frames: Optional[int] = None, median_width: int = 7, max_frames: int = 3000):
    """Short-form WhisperGenerationMixin.generate for ONE 3000-frame window (greedy, or beam search with
    num_beams > 1). Returns (final token sequence, language id); with alignment_heads (greedy only) also the
    token-level timestamps of return_token_timestamps=True (the top-level "token_timestamps": every pass's DTW
    times of the kept tokens, no seek offset; segments add seek * 0.01 s) and per pass the seek offset."""
    feats = np.asarray(feats, np.float32)

    def enc_at(seek):
        seg = segment_input(feats, seek, max_frames)
        if encoder_cache is not None and seek in encoder_cache:
            return encoder_cache[seek]
        e = model.encode(seg)
        if encoder_cache is not None:
            encoder_cache[seek] = e
        return e

    prompt = [g.sot]
    lang = None
    if g.multilingual:
        lang = language if language is not None else detect_language(model, enc_at(0), g)
        prompt.append(lang)
        if task is not None:
            prompt.append(g.transcribe if task == "transcribe" else g.translate)
        elif language is not None:
            prompt.append(g.transcribe)
    if not return_timestamps:
        prompt.append(g.notimestamps)
    P = len(prompt)
    max_new = max_new_tokens if max_new_tokens is not None else min(g.max_length + P, 448) - P
    seek, out = 0, []
    tts: List[float] = []
    pass_seeks: List[int] = []
    while seek < max_frames:
        xattn = {} if alignment_heads is not None else None
        if num_beams > 1:
            seq = beam_pass(model, enc_at(seek), prompt, max_new, g, return_timestamps, num_beams)
        else:
            seq = greedy_pass(model, enc_at(seek), prompt, max_new, g, return_timestamps, xattn=xattn)
        raw_ts = None
        if xattn is not None:
            rows = P + len(seq) - 1  # every fed position: the prompt and all generated tokens but the last
            w = np.stack([np.stack([xattn[t][l][h] for t in range(rows)]) for l, h in alignment_heads])
            nf = None if num_frames is None else num_frames - seek
            raw_ts = token_timestamps(w, P, nf, median_width)
        if seq and seq[-1] == g.eot:
            seq = seq[:-1]
        toks, off = retrieve_segment(seq, min(max_frames - seek, 3000), g.ts_begin)
        out += toks
        if raw_ts is not None:
            tts += [float(x) for x in raw_ts[P: P + len(toks)]]
            pass_seeks += [seek] * len(toks)
        seek += off
    if alignment_heads is not None:
        return out, lang, tts, pass_seeks
    return out, lang


def pass_criteria(model: WhisperOracle, feats: np.ndarray, g: GenCfg, prompt: Sequence[int], toks: Sequence[int],
                  seek: int = 0, use_ts: bool = True):
    """The temperature-fallback criteria of one greedy seek pass (generation_whisper.py:1243-1287) in fp32:
    (compression ratio of toks — _retrieve_compression_ratio, :1949-1956 —, average of log_softmax(processed
    scores)[token] over toks — _retrieve_avg_logprobs, :1958-1975 —, and WhisperNoSpeechDetection's softmax of the raw
    logits at the <|startoftranscript|> position at no_timestamps - 1 — logits_process.py:2091-2112). toks: the
    pass's generated tokens, EOS included, pads not (generate_with_fallback's cut, :1058-1066)."""
    import math
    import zlib

    length = int(math.log2(g.V) / 8) + 1
    raw = b"".join(int(t).to_bytes(length, "little") for t in toks)
    cr = len(raw) / len(zlib.compress(raw))
    feats = np.asarray(feats, np.float32)
    seg = np.zeros_like(feats)
    seg[:, : 3000 - seek] = feats[:, seek:]
    cache = model.new_cache(model.encode(seg))
    ids = list(prompt) + list(toks)
    lp, nsp = 0.0, None
    for t in range(len(ids) - 1):
        lg = model.decoder_step(int(ids[t]), cache)
        if t == 0:
            nsp = float(_softmax(lg.astype(np.float32))[g.notimestamps - 1])
        k = t - (len(prompt) - 1)
        if k >= 0:
            sc = process_logits(lg, list(toks[:k]), g, use_ts)
            fin = sc[np.isfinite(sc)]
            m = float(fin.max())
            lp += float(sc[int(toks[k])]) - (m + float(np.log(np.exp(fin - m).sum())))
    return cr, lp / max(1, len(toks)), nsp


def generate_batch_word(model: WhisperOracle, feats_list: Sequence[np.ndarray], g: GenCfg, alignment_heads,
                        num_frames: Sequence[int], task: Optional[str] = "transcribe", language: Optional[int] = None,
                        max_new_tokens: Optional[int] = None, median_width: int = 7, forced=None,
                        max_frames: Optional[Sequence[int]] = None):
    """generate(return_timestamps=True, return_token_timestamps=True) over a BATCH of windows (greedy), as the
    ASR pipeline's batched forward runs it: every seek pass decodes the batch's active rows together, and
    _extract_token_timestamps runs over the pass's padded batch -- rows that hit EOS keep being fed the pad
    token (= EOS) until the longest row ends, and those pad positions take part in the per-head standardization
    over tokens. ($TF/models/whisper/generation_whisper.py:241-400 over the batch of generate_with_fallback.)
    Returns per window (segment tokens, language id, token timestamps incl. the seek offsets).

    forced: optional per window (language id, [raw tokens of every seek pass]) of a device decode; the passes are
    then teacher-forced instead of decoded greedily (token-level timestamps of the device's own tokens, for inputs
    where bf16 took the other side of a greedy near-tie). max_frames: per window its feature frames (a long-form
    input's; default 3000)."""
    n = len(feats_list)
    feats_list = [np.asarray(f, np.float32) for f in feats_list]
    maxf = list(max_frames) if max_frames is not None else [3000] * n

    def enc_at(i, seek):
        return model.encode(segment_input(feats_list[i], seek, maxf[i]))

    langs: List[Optional[int]] = [None] * n
    prompts = []
    for i in range(n):
        prompt = [g.sot]
        if g.multilingual:
            if forced is not None:
                langs[i] = forced[i][0]
            else:
                langs[i] = language if language is not None else detect_language(model, enc_at(i, 0), g)
            prompt.append(langs[i])
            prompt.append(g.transcribe if (task or "transcribe") == "transcribe" else g.translate)
        prompts.append(prompt)
    P = len(prompts[0])
    max_new = max_new_tokens if max_new_tokens is not None else min(g.max_length + P, 448) - P
    seek = [0] * n
    outs: List[List[int]] = [[] for _ in range(n)]
    tts: List[List[float]] = [[] for _ in range(n)]
    npass = [0] * n
    while any(seek[i] < maxf[i] for i in range(n)):
        act = [i for i in range(n) if seek[i] < maxf[i]]
        seqs, xs, caches = {}, {}, {}
        for i in act:
            xs[i], co = {}, []
            if forced is not None:
                raw = list(forced[i][1][npass[i]])
                raw = raw[: raw.index(g.eot) + 1] if g.eot in raw else raw
                cache = model.new_cache(enc_at(i, seek[i]))
                cache["xattn"] = xs[i]
                for t in prompts[i] + raw[:-1]:
                    model.decoder_step(t, cache)
                seqs[i], caches[i] = raw, cache
            else:
                seqs[i] = greedy_pass(model, enc_at(i, seek[i]), prompts[i], max_new, g, True, xattn=xs[i],
                                      cache_out=co)
                caches[i] = co[0]
            npass[i] += 1
        L = max(len(seqs[i]) for i in act)
        rows = P + L - 1
        for i in act:  # pad rows: the finished row is fed EOS (its own last token, then the pad token)
            for _ in range(L - len(seqs[i])):
                model.decoder_step(g.eot, caches[i])
            w = np.stack([np.stack([xs[i][t][l][h] for t in range(rows)]) for l, h in alignment_heads])
            raw_ts = token_timestamps(w, P, num_frames[i] - seek[i], median_width)
            seq = seqs[i][:-1] if seqs[i][-1] == g.eot else seqs[i]
            toks, off = retrieve_segment(seq, min(maxf[i] - seek[i], 3000), g.ts_begin)
            outs[i] += toks
            o = np.float32(seek[i] * 0.02 / 2)
            tts[i] += [float(np.float32(x) + o) for x in raw_ts[P: P + len(toks)]]
            seek[i] += off
    return [(outs[i], langs[i], tts[i]) for i in range(n)]


# ----------------------------------------------------------------------------- tolerant greedy replay
def decision_ok(scores: np.ndarray, sampled: Sequence[int], g: GenCfg, use_ts: bool, tok: int, tau: float) -> bool:
    """Is `tok` a greedy choice of the f32 reference at this step within tolerance `tau` (in logits)?

    The exact argmax of the processed scores always is. Otherwise `tok` must trail the f32 choice by at most tau on
    the processed scores; or, when the timestamp rule (timestamp log-prob mass vs the best text log-prob) is itself
    within tau of flipping, trail the best token of its own class (timestamp / text) by at most tau."""
    s = process_logits(scores, sampled, g, use_ts)
    best = int(np.argmax(s))
    if tok == best or (np.isfinite(s[tok]) and s[tok] >= s[best] - tau):
        return True
    if use_ts:
        pre = process_logits_no_rule(scores, sampled, g)
        tb = g.ts_begin
        if abs(_ts_rule_margin(pre, tb)) <= tau and np.isfinite(pre[tok]):
            cls = pre[tb:] if tok >= tb else pre[:tb]
            return bool(pre[tok] >= np.max(cls) - tau)
    return False


def process_logits_no_rule(scores: np.ndarray, sampled: Sequence[int], g: GenCfg) -> np.ndarray:
    """process_logits with timestamps on, minus the final log-sum-exp rule."""
    s = scores.astype(np.float32).copy()
    n = len(sampled)
    if n == 0 and g.begin_suppress:
        s[g.begin_suppress] = -np.inf
    if g.suppress:
        s[g.suppress] = -np.inf
    tb = g.ts_begin
    s[g.notimestamps] = -np.inf
    last_ts = n >= 1 and sampled[-1] >= tb
    pen_ts = n < 2 or sampled[-2] >= tb
    if last_ts:
        if pen_ts:
            s[tb:] = -np.inf
        else:
            s[: g.eot] = -np.inf
    tss = [t for t in sampled if t >= tb]
    if tss:
        tl = tss[-1] if (last_ts and not pen_ts) else tss[-1] + 1
        s[tb:tl] = -np.inf
    if n == 0:
        s[:tb] = -np.inf
        if g.mit is not None:
            s[tb + g.mit + 1:] = -np.inf
    return s


def replay_generate(model: WhisperOracle, feats: np.ndarray, g: GenCfg, passes: Sequence[Sequence[int]],
                    lang: Optional[int], task: Optional[str] = "transcribe", return_timestamps: bool = True,
                    max_new_tokens: Optional[int] = None, tau: float = 0.3, mx: bool = False,
                    max_frames: int = 3000, prefixes: Optional[Sequence] = None) -> dict:
    """Follow a device decode of ONE window (its raw per-seek-pass token lists and detected language) through the
    f32 reference, checking every decision with decision_ok. Returns {"ok", "decisions", "exact", "first_bad"}.
    mx: the reference encoder is encode_mx (config 5's MX fp8 projections). max_frames: the input's feature frames
    (long-form). prefixes: per pass None or (tokens, pads) — the condition_on_prev_tokens prompt the device fed ahead of
    the init tokens (its pad tokens left out: new_cache(pos0=pads))."""
    feats = np.asarray(feats, np.float32)
    stats = {"ok": True, "decisions": 0, "exact": 0, "first_bad": None}

    def enc_at(seek):
        seg = segment_input(feats, seek, max_frames)
        return model.encode_mx(seg) if mx else model.encode(seg)

    def check(scores, sampled, tok, use_ts):
        stats["decisions"] += 1
        if int(np.argmax(process_logits(scores, sampled, g, use_ts))) == tok:
            stats["exact"] += 1
            return
        if not decision_ok(scores, sampled, g, use_ts, tok, tau) and stats["first_bad"] is None:
            stats["ok"] = False
            stats["first_bad"] = (len(sampled), tok, sampled[-5:])

    prompt = [g.sot]
    if g.multilingual:
        if lang is None:
            raise ValueError("multilingual replay needs the device's language id")
        cache = model.new_cache(enc_at(0))
        lg = model.decoder_step(g.sot, cache)
        ml = np.full_like(lg, -np.inf)
        ml[g.lang_begin: g.lang_begin + g.n_lang] = lg[g.lang_begin: g.lang_begin + g.n_lang]
        stats["decisions"] += 1
        if int(np.argmax(ml)) == lang:
            stats["exact"] += 1
        elif not ml[lang] >= np.max(ml) - tau:
            stats["ok"], stats["first_bad"] = False, ("language", lang, int(np.argmax(ml)))
        prompt.append(lang)
        if task is not None:
            prompt.append(g.transcribe if task == "transcribe" else g.translate)
    if not return_timestamps:
        prompt.append(g.notimestamps)
    P = len(prompt)
    max_new = max_new_tokens if max_new_tokens is not None else min(g.max_length + P, 448) - P
    seek = 0
    for k, seq_raw in enumerate(passes):
        if seek >= max_frames:
            stats["ok"], stats["first_bad"] = False, ("extra pass", seek, None)
            break
        pf = prefixes[k] if prefixes is not None else None
        toks_p, pads = (list(pf[0][pf[1]:]), int(pf[1])) if pf is not None else ([], 0)
        cache = model.new_cache(enc_at(seek), pos0=pads)
        for t in toks_p + prompt[:-1]:
            model.decoder_step(t, cache)
        logits = model.decoder_step(prompt[-1], cache)
        mn = max_new
        if pf is not None and max_new_tokens is None:
            mn = min(g.max_length + P + len(pf[0]), 448) - P - len(pf[0])
        out: List[int] = []
        for tok in seq_raw:
            check(logits, out, int(tok), return_timestamps)
            out.append(int(tok))
            if tok == g.eot or len(out) >= mn:
                break
            logits = model.decoder_step(int(tok), cache)
        seq = out[:-1] if out and out[-1] == g.eot else out
        _, off = retrieve_segment(seq, min(max_frames - seek, 3000), g.ts_begin)
        seek += off
    if seek < max_frames:
        stats["ok"], stats["first_bad"] = False, ("missing pass", seek, None)
    return stats

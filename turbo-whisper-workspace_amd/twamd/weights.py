"""Parameter schema, seeded synthetic parameters and the HBM packing of a Whisper model.

Names follow the Hugging Face `WhisperForConditionalGeneration` state dict (the module tree the
reference loads through `transformers.pipeline`, /root/reference/vocalis/core/audio_pipeline.py:195-200;
$TF/models/whisper/modeling_whisper.py). Synthetic parameters are defined per tensor name by
`synth_spec` and produced on the device by `tw_fill_synth` (csrc/tw_runtime.hip); the oracle and the
golden-vector script regenerate the identical values in numpy.

Packed layout in HBM (bf16 matrices row-major [out][in], f32 vectors):
  encoder: conv1_w [D][kpad1] (k = j*n_mels + c), conv2_w [D][3D] (k = j*D + c), pos f32 [1500][D],
           per layer wqkv [3D][D] (q rows and bias pre-multiplied by 0.125), wo, w1 [F][D], w2 [D][F]
  decoder: emb [V][D] (= tied proj_out), pos [448][D], per layer self wqkv / wo, cross wq / wo,
           w1, w2; all layers' cross K/V projections stacked in one [L*2*D][D] matrix so the
           cross-attention cache of a window is ONE GEMM after the encoder.
"""
from __future__ import annotations

import dataclasses
import os
import zlib
from typing import Dict, List, Optional, Tuple

import torch

from . import _lib
from .config import WhisperDims


def param_shapes(d: WhisperDims) -> List[Tuple[str, Tuple[int, ...]]]:
    """Ordered (name, shape) of every parameter (proj_out is tied to decoder.embed_tokens)."""
    D, F = d.d_model, d.ffn
    out: List[Tuple[str, Tuple[int, ...]]] = [
        ("model.encoder.conv1.weight", (D, d.n_mels, 3)),
        ("model.encoder.conv1.bias", (D,)),
        ("model.encoder.conv2.weight", (D, D, 3)),
        ("model.encoder.conv2.bias", (D,)),
        ("model.encoder.embed_positions.weight", (d.max_source_positions, D)),
    ]

    def attn(prefix: str) -> None:
        out.extend([
            (f"{prefix}.k_proj.weight", (D, D)),
            (f"{prefix}.v_proj.weight", (D, D)), (f"{prefix}.v_proj.bias", (D,)),
            (f"{prefix}.q_proj.weight", (D, D)), (f"{prefix}.q_proj.bias", (D,)),
            (f"{prefix}.out_proj.weight", (D, D)), (f"{prefix}.out_proj.bias", (D,)),
        ])

    def ln(prefix: str) -> None:
        out.extend([(f"{prefix}.weight", (D,)), (f"{prefix}.bias", (D,))])

    def mlp(prefix: str) -> None:
        out.extend([(f"{prefix}.fc1.weight", (F, D)), (f"{prefix}.fc1.bias", (F,)),
                    (f"{prefix}.fc2.weight", (D, F)), (f"{prefix}.fc2.bias", (D,))])

    for i in range(d.encoder_layers):
        p = f"model.encoder.layers.{i}"
        attn(f"{p}.self_attn")
        ln(f"{p}.self_attn_layer_norm")
        mlp(p)
        ln(f"{p}.final_layer_norm")
    ln("model.encoder.layer_norm")
    out.append(("model.decoder.embed_tokens.weight", (d.vocab, D)))
    out.append(("model.decoder.embed_positions.weight", (d.max_target_positions, D)))
    for i in range(d.decoder_layers):
        p = f"model.decoder.layers.{i}"
        attn(f"{p}.self_attn")
        ln(f"{p}.self_attn_layer_norm")
        attn(f"{p}.encoder_attn")
        ln(f"{p}.encoder_attn_layer_norm")
        mlp(p)
        ln(f"{p}.final_layer_norm")
    ln("model.decoder.layer_norm")
    return out


def synth_spec(name: str, shape: Tuple[int, ...], d: WhisperDims) -> Tuple[int, float, float]:
    """(tensor_id, scale, offset) of the seeded uniform(-1,1)*scale+offset parameter `name`.

    Scales keep activations O(1) through the stack (uniform std = scale/sqrt(3)); the token embedding
    std is 2/sqrt(D) (logit std ~2): wide enough that greedy decoding is not dominated by near-ties,
    narrow enough that the embedding of the last token does not dominate the residual stream (which
    makes a random decoder repeat one token forever) — it yields timestamp pairs, text runs and
    multi-pass seeks, exercising the whole generate() path.
    """
    tid = zlib.crc32(name.encode()) & 0xFFFFFFFF
    if "layer_norm" in name:
        return (tid, 0.2, 1.0) if name.endswith("weight") else (tid, 0.1, 0.0)
    if name.endswith("embed_tokens.weight"):
        return tid, (3.0 ** 0.5) * 2.0 / (d.d_model ** 0.5), 0.0
    if name.endswith("embed_positions.weight"):
        return tid, 0.5, 0.0
    if name.endswith("bias"):
        return tid, 0.05, 0.0
    fan_in = 1
    for s in shape[1:]:
        fan_in *= s
    return tid, (3.0 / fan_in) ** 0.5, 0.0


@dataclasses.dataclass
class EncoderLayerW:
    ln1_g: torch.Tensor
    ln1_b: torch.Tensor
    wqkv: torch.Tensor
    bqkv: torch.Tensor
    wo: torch.Tensor
    bo: torch.Tensor
    ln2_g: torch.Tensor
    ln2_b: torch.Tensor
    w1: torch.Tensor
    b1: torch.Tensor
    w2: torch.Tensor
    b2: torch.Tensor


@dataclasses.dataclass
class DecoderLayerW:
    ln1_g: torch.Tensor
    ln1_b: torch.Tensor
    wqkv: torch.Tensor
    bqkv: torch.Tensor
    wo: torch.Tensor
    bo: torch.Tensor
    ln2_g: torch.Tensor
    ln2_b: torch.Tensor
    wq_x: torch.Tensor
    bq_x: torch.Tensor
    wo_x: torch.Tensor
    bo_x: torch.Tensor
    ln3_g: torch.Tensor
    ln3_b: torch.Tensor
    w1: torch.Tensor
    b1: torch.Tensor
    w2: torch.Tensor
    b2: torch.Tensor


@dataclasses.dataclass
class PackedWeights:
    dims: WhisperDims
    kpad1: int
    conv1_w: torch.Tensor
    conv1_b: torch.Tensor
    conv2_w: torch.Tensor
    conv2_b: torch.Tensor
    pos_enc: torch.Tensor
    enc: List[EncoderLayerW]
    enc_ln_g: torch.Tensor
    enc_ln_b: torch.Tensor
    emb: torch.Tensor
    pos_dec: torch.Tensor
    dec: List[DecoderLayerW]
    dec_ln_g: torch.Tensor
    dec_ln_b: torch.Tensor
    wkv_x: torch.Tensor  # [L*2*D][D]
    bkv_x: torch.Tensor  # [L*2*D]

    def nbytes(self) -> int:
        n = 0
        for f in dataclasses.fields(self):
            v = getattr(self, f.name)
            if isinstance(v, torch.Tensor):
                n += v.numel() * v.element_size()
            elif isinstance(v, list):
                for lw in v:
                    for g in dataclasses.fields(lw):
                        t = getattr(lw, g.name)
                        n += t.numel() * t.element_size()
        return n


def synth_state_dict(d: WhisperDims, seed: int, device: str = "cuda") -> Dict[str, torch.Tensor]:
    """Generate every parameter on the device with tw_fill_synth (bf16 matrices, f32 vectors)."""
    sd: Dict[str, torch.Tensor] = {}
    stream = _lib.stream_handle()
    for name, shape in param_shapes(d):
        tid, scale, offset = synth_spec(name, shape, d)
        as_f32 = len(shape) == 1
        t = torch.empty(shape, dtype=torch.float32 if as_f32 else torch.bfloat16, device=device)
        _lib.call("tw_fill_synth", t.data_ptr(), t.numel(), seed, tid, scale, offset, int(as_f32), stream)
        sd[name] = t
    return sd


def load_checkpoint_state_dict(path: str, d: WhisperDims, device: str = "cuda",
                               dtype: torch.dtype = torch.bfloat16) -> Dict[str, torch.Tensor]:
    """Read a local Hugging Face Whisper checkpoint directory (*.safetensors; no network): matrices as `dtype`,
    vectors f32."""
    from safetensors.torch import load_file

    files = sorted(f for f in os.listdir(path) if f.endswith(".safetensors"))
    if not files:
        raise FileNotFoundError(f"no *.safetensors in {path}")
    sd: Dict[str, torch.Tensor] = {}
    for f in files:
        for k, v in load_file(os.path.join(path, f)).items():
            if k.startswith("proj_out"):
                continue
            sd[k] = v
    out = {}
    for name, shape in param_shapes(d):
        if name not in sd:
            raise KeyError(f"checkpoint {path} lacks {name}")
        v = sd[name]
        if tuple(v.shape) != tuple(shape):
            raise ValueError(f"{name}: shape {tuple(v.shape)} != {shape}")
        out[name] = v.to(device=device, dtype=torch.float32 if len(shape) == 1 else dtype)
    return out


def pack(sd: Dict[str, torch.Tensor], d: WhisperDims, dtype: torch.dtype = torch.bfloat16) -> PackedWeights:
    """Repack a state dict (matrices / f32 vectors on the device) into the engine layout, matrices as `dtype` (bf16:
    the bf16 engine; f32: the fp32 path, WhisperEngineF32). The q scale 0.125 is a power of two: exact in both.

    Runs once at model load (torch ops used as device-memory plumbing, not on the hot path)."""
    D, F, M = d.d_model, d.ffn, d.n_mels
    dev = sd["model.encoder.conv1.bias"].device
    bf, f32 = dtype, torch.float32

    def mat(n):
        return sd[n].to(bf).contiguous()

    def vec(n):
        return sd[n].to(f32).contiguous()

    kpad1 = (3 * M + 63) // 64 * 64
    c1 = sd["model.encoder.conv1.weight"].to(bf).permute(0, 2, 1).reshape(D, 3 * M)
    conv1_w = torch.zeros(D, kpad1, dtype=bf, device=dev)
    conv1_w[:, : 3 * M] = c1
    conv2_w = sd["model.encoder.conv2.weight"].to(bf).permute(0, 2, 1).reshape(D, 3 * D).contiguous()
    zero_d = torch.zeros(D, dtype=f32, device=dev)

    def qkv(prefix):
        w = torch.cat([sd[f"{prefix}.q_proj.weight"].to(bf) * 0.125, sd[f"{prefix}.k_proj.weight"].to(bf),
                       sd[f"{prefix}.v_proj.weight"].to(bf)], 0).contiguous()
        b = torch.cat([vec(f"{prefix}.q_proj.bias") * 0.125, zero_d, vec(f"{prefix}.v_proj.bias")]).contiguous()
        return w, b

    enc = []
    for i in range(d.encoder_layers):
        p = f"model.encoder.layers.{i}"
        w, b = qkv(f"{p}.self_attn")
        enc.append(EncoderLayerW(
            vec(f"{p}.self_attn_layer_norm.weight"), vec(f"{p}.self_attn_layer_norm.bias"), w, b,
            mat(f"{p}.self_attn.out_proj.weight"), vec(f"{p}.self_attn.out_proj.bias"),
            vec(f"{p}.final_layer_norm.weight"), vec(f"{p}.final_layer_norm.bias"),
            mat(f"{p}.fc1.weight"), vec(f"{p}.fc1.bias"), mat(f"{p}.fc2.weight"), vec(f"{p}.fc2.bias")))
    dec = []
    kv_w, kv_b = [], []
    for i in range(d.decoder_layers):
        p = f"model.decoder.layers.{i}"
        w, b = qkv(f"{p}.self_attn")
        x = f"{p}.encoder_attn"
        dec.append(DecoderLayerW(
            vec(f"{p}.self_attn_layer_norm.weight"), vec(f"{p}.self_attn_layer_norm.bias"), w, b,
            mat(f"{p}.self_attn.out_proj.weight"), vec(f"{p}.self_attn.out_proj.bias"),
            vec(f"{p}.encoder_attn_layer_norm.weight"), vec(f"{p}.encoder_attn_layer_norm.bias"),
            (sd[f"{x}.q_proj.weight"].to(bf) * 0.125).contiguous(), vec(f"{x}.q_proj.bias") * 0.125,
            mat(f"{x}.out_proj.weight"), vec(f"{x}.out_proj.bias"),
            vec(f"{p}.final_layer_norm.weight"), vec(f"{p}.final_layer_norm.bias"),
            mat(f"{p}.fc1.weight"), vec(f"{p}.fc1.bias"), mat(f"{p}.fc2.weight"), vec(f"{p}.fc2.bias")))
        kv_w += [mat(f"{x}.k_proj.weight"), mat(f"{x}.v_proj.weight")]
        kv_b += [zero_d, vec(f"{x}.v_proj.bias")]
    return PackedWeights(
        dims=d, kpad1=kpad1, conv1_w=conv1_w, conv1_b=vec("model.encoder.conv1.bias"), conv2_w=conv2_w,
        conv2_b=vec("model.encoder.conv2.bias"),
        pos_enc=sd["model.encoder.embed_positions.weight"].to(f32).contiguous(), enc=enc,
        enc_ln_g=vec("model.encoder.layer_norm.weight"), enc_ln_b=vec("model.encoder.layer_norm.bias"),
        emb=mat("model.decoder.embed_tokens.weight"), pos_dec=mat("model.decoder.embed_positions.weight"), dec=dec,
        dec_ln_g=vec("model.decoder.layer_norm.weight"), dec_ln_b=vec("model.decoder.layer_norm.bias"),
        wkv_x=torch.cat(kv_w, 0).contiguous(), bkv_x=torch.cat(kv_b).contiguous())


def build_weights(d: WhisperDims, seed: Optional[int] = 1234, checkpoint: Optional[str] = None,
                  dtype: torch.dtype = torch.bfloat16) -> PackedWeights:
    """dtype: the matrices' type (bf16, or f32 for the fp32 path; the synthetic matrices are bf16-valued either way,
    the values transformers' fp32 goldens were made with)."""
    sd = load_checkpoint_state_dict(checkpoint, d, dtype=dtype) if checkpoint else synth_state_dict(d, seed)
    pw = pack(sd, d, dtype)
    del sd
    return pw

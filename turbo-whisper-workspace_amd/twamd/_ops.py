"""The torch.ops.tw.* custom operators (csrc/torch_ops.cpp, built as libtwhip_torch.so next to libtwhip.so).

Loaded once with torch.ops.load_library; there is no fallback: a missing library raises, as _lib.load() does for the
C-ABI library. The ops launch the same HIP kernels as the C-ABI calls, on torch's current stream, with Meta (shape)
implementations for FakeTensor tracing. The engine's encoder path (conv stem GEMMs, LayerNorms, q/k/v/o and FFN
projections, the attention core, the cross-K/V projection) and the log-mel run through them."""
from __future__ import annotations

import os

import torch

from . import _lib

TORCH_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libtwhip_torch.so")
_loaded = False


def load():
    """torch.ops.tw, with the operator library loaded (after the C-ABI library it links)."""
    global _loaded
    if not _loaded:
        _lib.load()
        if not os.path.exists(TORCH_LIB_PATH):
            raise _lib.TwError(f"torch operator library not built: {TORCH_LIB_PATH} "
                               "(run `make -C turbo-whisper-workspace_amd/csrc`)")
        torch.ops.load_library(TORCH_LIB_PATH)
        _loaded = True
    return torch.ops.tw


OPS = ("logmel", "logmel_out", "gemm_bf16", "gemm_bf16_out", "attn_encoder", "attn_encoder_out", "layernorm",
       "layernorm_out", "gemv_packed_out", "resid_layernorm_packed_", "attn_decode_self_", "attn_decode_cross_out",
       "logits_select_")

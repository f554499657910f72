"""ctypes binding of libtwhip.so, the C-ABI declared in include/tw_whisper.h and include/tw_audio.h.

The library must be built (`make -C turbo-whisper-workspace_amd/csrc`, or `__graft_entry__.build()`).
There is deliberately no fallback: if the HIP library is missing every engine entry point raises.
torch is imported first so that libtwhip.so binds to the HIP runtime torch already loaded
(both carry SONAME libamdhip64.so.7; the dynamic linker reuses the loaded one).
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (load torch's HIP runtime before ours)

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libtwhip.so")
# the same library built with -DTW_DEBUG=1 (`make -C turbo-whisper-workspace_amd/csrc debug`): C-ABI contract checks
DEBUG_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libtwhip_dbg.so")

TW_EPI_BF16 = 0
TW_EPI_GELU_BF16 = 1
TW_EPI_RESID_F32 = 2
TW_EPI_GELU_POS_F32 = 3
TW_EPI_F32 = 4
TW_EPI_CROSSKV = 5
TW_EPI_GELU_PACKED = 6
TW_EPI_GELU_MX = 7
TW_EPI_GELU_F32 = 8
TW_EPI_PARTIAL_F32 = 100

TW_SELECT_CHUNKS = 16
TW_SELECT_WS_PER_ROW = 128
TW_STATE_STRIDE = 8
TW_ST_NGEN, TW_ST_LAST, TW_ST_PENULT, TW_ST_LASTTS, TW_ST_FINISHED, TW_ST_LANG = 0, 1, 2, 3, 4, 5
TW_ST_SUMLP, TW_ST_NOSPEECH = 6, 7  # f32 bits (tw_logits_sample / tw_token_prob)

# every symbol include/tw_whisper.h + include/tw_audio.h declare (tests check the .so exports all of them)
EXPORTED = (
    "tw_version", "tw_last_error", "tw_fill_synth", "tw_f32_to_bf16", "tw_logmel", "tw_im2col_conv1",
    "tw_im2col_conv2", "tw_gemm_bf16", "tw_layernorm", "tw_attn_encoder", "tw_attn_decode_self",
    "tw_attn_decode_cross", "tw_embed_decoder", "tw_logits_select", "tw_gemm_bf16_partial", "tw_resid_layernorm",
    "tw_gemm_set_variant", "tw_attn_set_variant",
    "tw_dtw", "tw_attn_decode_cross_probs", "tw_attn_decode_cross_grouped", "tw_attn_decode_cross_grouped_ws_bytes", "tw_attn_decode_self_tab", "tw_beam_workspace_bytes", "tw_beam_step", "tw_kv_reorder", "tw_pack_weight", "tw_gemv_packed", "tw_resid_layernorm_packed", "tw_flac_probe", "tw_flac_decode", "tw_resample_pcm_i32", "tw_resample_pcm_f32",
    "tw_gemm_mx", "tw_quant_mx", "tw_layernorm_mx", "tw_attn_encoder_mx", "tw_gemm_mx_set_variant", "tw_logits_select_embed",
    "tw_attn_set_lds_pad", "tw_logits_sample", "tw_token_prob", "tw_g711_decode", "tw_ima_adpcm_wav_decode",
    "tw_ms_adpcm_wav_decode", "tw_ima_qt_decode", "tw_alac_parse_cookie", "tw_alac_decode",
    "tw_kv_tab_check", "tw_debug_build", "tw_resid_layernorm_packed_to", "tw_conv2_gemm",
    "tw_logmel_long", "tw_im2col_conv1_long", "tw_attn_decode_self_masked", "tw_attn_decode_self_tab_masked",
    "tw_gemv_set_wide_slices", "tw_vorbis_probe", "tw_vorbis_decode", "tw_vorbis_imdct",
    "tw_layernorm_set_lds_pad", "tw_gemv_set_variant",
    "tw_gemm_f32", "tw_layernorm_f32", "tw_im2col_conv1_f32", "tw_im2col_conv2_f32", "tw_embed_decoder_f32",
    "tw_attn_encoder_f32", "tw_attn_decode_self_f32", "tw_attn_decode_cross_f32", "tw_gemm_set_epilogue",
    "tw_gemm_set_persistent_grid", "tw_mp3_probe", "tw_mp3_decode", "tw_aac_parse_asc", "tw_aac_decode_raw",
    "tw_aac_adts_probe", "tw_aac_adts_decode", "tw_dec_fused", "tw_dec_fused_sync_bytes", "tw_dec_fused_supported",
    "tw_dec_fused_set_grid", "tw_dec_fused_set_acquire", "tw_dec_fused_set_probe", "tw_dec_fused_grid",
    "tw_dec_fused_xpart_bytes",
)


class TwSelectParams(ctypes.Structure):
    _fields_ = [
        ("V", ctypes.c_int32), ("eos", ctypes.c_int32), ("pad", ctypes.c_int32), ("ts_begin", ctypes.c_int32),
        ("no_timestamps", ctypes.c_int32), ("max_initial_ts", ctypes.c_int32), ("use_timestamps", ctypes.c_int32),
        ("max_new", ctypes.c_int32), ("mode", ctypes.c_int32), ("lo", ctypes.c_int32), ("hi", ctypes.c_int32),
        ("n_begin_suppress", ctypes.c_int32), ("begin_suppress", ctypes.c_int32 * 8),
    ]


class TwBeamParams(ctypes.Structure):
    _fields_ = [("num_beams", ctypes.c_int32), ("max_new", ctypes.c_int32), ("length_penalty", ctypes.c_float),
                ("ld_tokens", ctypes.c_int32)]


class TwBeamState(ctypes.Structure):
    _fields_ = [("run_score", ctypes.c_void_p), ("fin_score", ctypes.c_void_p), ("fin_flag", ctypes.c_void_p),
                ("fin_len", ctypes.c_void_p), ("fin_tokens", ctypes.c_void_p), ("win", ctypes.c_void_p),
                ("src_rows", ctypes.c_void_p), ("kv_tab", ctypes.c_void_p), ("fin_tab", ctypes.c_void_p),
                ("run_lp", ctypes.c_void_p), ("fin_lp", ctypes.c_void_p)]


class TwFlacInfo(ctypes.Structure):
    _fields_ = [
        ("sample_rate", ctypes.c_int32), ("channels", ctypes.c_int32), ("bits_per_sample", ctypes.c_int32),
        ("min_blocksize", ctypes.c_int32), ("max_blocksize", ctypes.c_int32), ("total_from_frames", ctypes.c_int32),
        ("total_samples", ctypes.c_int64), ("audio_offset", ctypes.c_int64), ("md5", ctypes.c_uint8 * 16),
    ]


class TwVorbisInfo(ctypes.Structure):
    _fields_ = [
        ("sample_rate", ctypes.c_int32), ("channels", ctypes.c_int32), ("blocksize0", ctypes.c_int32),
        ("blocksize1", ctypes.c_int32), ("total_samples", ctypes.c_int64),
    ]


class TwMp3Info(ctypes.Structure):
    _fields_ = [
        ("sample_rate", ctypes.c_int32), ("channels", ctypes.c_int32), ("version", ctypes.c_int32),
        ("bitrate_kbps", ctypes.c_int32), ("total_samples", ctypes.c_int64), ("n_frames", ctypes.c_int64),
        ("skip_samples", ctypes.c_int64), ("samples_per_frame", ctypes.c_int32), ("enc_delay", ctypes.c_int32),
        ("enc_padding", ctypes.c_int32), ("flags", ctypes.c_int32), ("layer", ctypes.c_int32),
    ]


class TwAlacInfo(ctypes.Structure):
    _fields_ = [
        ("sample_rate", ctypes.c_int32), ("channels", ctypes.c_int32), ("bit_depth", ctypes.c_int32),
        ("frame_length", ctypes.c_int32), ("pb", ctypes.c_int32), ("mb", ctypes.c_int32), ("kb", ctypes.c_int32),
    ]


class TwAacInfo(ctypes.Structure):
    _fields_ = [
        ("sample_rate", ctypes.c_int32), ("channels", ctypes.c_int32), ("object_type", ctypes.c_int32),
        ("frame_length", ctypes.c_int32), ("n_frames", ctypes.c_int64), ("total_samples", ctypes.c_int64),
    ]


class TwError(RuntimeError):
    pass


_P = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_long
_F = ctypes.c_float
_U64 = ctypes.c_uint64
_U32 = ctypes.c_uint32

_SIGS = {
    "tw_version": ([], _I),
    "tw_last_error": ([], ctypes.c_char_p),
    "tw_fill_synth": ([_P, _L, _U64, _U32, _F, _F, _I, _P], _I),
    "tw_f32_to_bf16": ([_P, _P, _L, _F, _P], _I),
    "tw_logmel": ([_P, _I, _P, _P, _P, _I, _P, _P, _P], _I),
    "tw_im2col_conv1": ([_P, _I, _P, _P, _I, _I, _P, _P], _I),
    "tw_im2col_conv1_long": ([_P, _I, _L, _P, _P, _P, _I, _I, _P, _P], _I),
    "tw_logmel_long": ([_P, _L, _P, _P, _P, _I, _P, _L, _P, _P], _I),
    "tw_im2col_conv2": ([_P, _I, _I, _P, _P], _I),
    "tw_conv2_gemm": ([_P, _I, _I, _P, _P, _P, _P, _P], _I),
    "tw_gemm_bf16": ([_P, _P, _I, _I, _I, _I, _I, _I, _P, _I, _P, _P, _I, _P, _P], _I),
    "tw_layernorm": ([_P, _P, _P, _I, _I, _F, _P, _P], _I),
    "tw_gemm_set_epilogue": ([_I], _I),
    "tw_gemm_set_persistent_grid": ([_I], _I),
    "tw_gemm_f32": ([_P, _P, _I, _I, _I, _I, _I, _I, _P, _I, _P, _P, _I, _P, _P], _I),
    "tw_layernorm_f32": ([_P, _P, _P, _I, _I, _F, _P, _P], _I),
    "tw_im2col_conv1_f32": ([_P, _I, _L, _P, _P, _P, _I, _I, _P, _P], _I),
    "tw_im2col_conv2_f32": ([_P, _I, _I, _P, _P], _I),
    "tw_embed_decoder_f32": ([_P, _P, _P, _P, _I, _I, _P, _P], _I),
    "tw_attn_encoder_f32": ([_P, _I, _I, _I, _P, _P], _I),
    "tw_attn_decode_self_f32": ([_P, _I, _I, _I, _P, _P, _P, _P, _I, _P, _P, _P], _I),
    "tw_attn_decode_cross_f32": ([_P, _I, _I, _I, _I, _P, _P, _P, _P, _U32, _I, _I, _P, _I, _I, _P], _I),
    "tw_gemm_mx": ([_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _P, _I, _P, _P, _I, _P], _I),
    "tw_quant_mx": ([_P, _I, _I, _I, _P, _P, _I, _P], _I),
    "tw_attn_encoder_mx": ([_P, _I, _I, _I, _P, _P, _I, _P], _I),
    "tw_layernorm_mx": ([_P, _P, _P, _I, _I, _F, _P, _P, _I, _P], _I),
    "tw_attn_encoder": ([_P, _I, _I, _I, _P, _P], _I),
    "tw_attn_decode_self": ([_P, _I, _I, _I, _P, _P, _P, _P, _P], _I),
    "tw_attn_decode_self_masked": ([_P, _I, _I, _I, _P, _P, _P, _P, _P, _P], _I),
    "tw_attn_decode_cross": ([_P, _I, _I, _I, _I, _P, _P, _P, _P], _I),
    "tw_attn_decode_cross_grouped": ([_P, _I, _I, _I, _I, _P, _I, _I, _P, _P, _P, _P], _I),
    "tw_embed_decoder": ([_P, _P, _P, _P, _I, _I, _P, _P], _I),
    "tw_logits_select": ([_P, _I, _I, _P, ctypes.POINTER(TwSelectParams), _P, _P, _I, _P, _P, _P, _P], _I),
    "tw_logits_sample": ([_P, _I, _I, _P, ctypes.POINTER(TwSelectParams), ctypes.c_float, _I, ctypes.c_uint64, _P, _P,
                          _P, _I, _P, _P, _P], _I),
    "tw_token_prob": ([_P, _I, _I, _I, _I, _P, _P], _I),
    "tw_gemm_bf16_partial": ([_P, _P, _I, _I, _I, _I, _I, _I, _P, _I, _P], _I),
    "tw_gemv_set_wide_slices": ([_I], _I),
    "tw_gemv_set_variant": ([_I], _I),
    "tw_gemm_set_variant": ([_I], _I),
    "tw_gemm_mx_set_variant": ([_I], _I),
    "tw_logits_select_embed": ([_P, _I, _I, _P, ctypes.POINTER(TwSelectParams), _P, _P, _I, _P, _P, _P, _P, _P, _I,
                                _I, _P, _P, _P, _F, _P, _I, _P], _I),
    "tw_attn_set_variant": ([_I], _I),
    "tw_attn_set_lds_pad": ([_I], _I),
    "tw_resid_layernorm": ([_P, _P, _I, _P, _P, _P, _I, _I, _F, _P, _P], _I),
    "tw_dtw": ([_P, _I, _I, _P, _P, _P], _I),
    "tw_attn_decode_cross_probs": ([_P, _I, _I, _I, _I, _P, _P, _P, _P, _U32, _I, _I, _P, _I, _I, _P], _I),
    "tw_beam_workspace_bytes": ([_I], ctypes.c_size_t),
    "tw_attn_decode_cross_grouped_ws_bytes": ([_I, _I], ctypes.c_size_t),
    "tw_attn_decode_self_tab": ([_P, _I, _I, _I, _P, _P, _P, _P, _I, _P, _P], _I),
    "tw_attn_decode_self_tab_masked": ([_P, _I, _I, _I, _P, _P, _P, _P, _I, _P, _P, _P], _I),
    "tw_kv_tab_check": ([_P, _P, _I, _I, _I, _P, _P], _I),
    "tw_debug_build": ([], _I),
    "tw_beam_step": ([_P, _I, _I, _P, ctypes.POINTER(TwSelectParams), ctypes.POINTER(TwBeamParams),
                      ctypes.POINTER(TwBeamState), _P, _P, _P, _P, _P, _P], _I),
    "tw_kv_reorder": ([_P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _P, _P], _I),
    "tw_pack_weight": ([_P, _I, _I, _I, _P, _P], _I),
    "tw_gemv_packed": ([_P, _I, _I, _P, _I, _I, _I, _I, _P, _I, _P, _I, _P], _I),
    "tw_resid_layernorm_packed": ([_P, _P, _I, _P, _P, _P, _I, _I, _F, _P, _P], _I),
    "tw_resid_layernorm_packed_to": ([_P, _P, _P, _I, _P, _P, _P, _I, _I, _F, _P, _P], _I),
    "tw_flac_probe": ([_P, ctypes.c_int64, ctypes.POINTER(TwFlacInfo)], _I),
    "tw_flac_decode": ([_P, ctypes.c_int64, _P, ctypes.c_int64, _I, ctypes.POINTER(ctypes.c_int64)], _I),
    "tw_g711_decode": ([_P, ctypes.c_int64, _I, _P], _I),
    "tw_vorbis_probe": ([_P, ctypes.c_int64, ctypes.POINTER(TwVorbisInfo)], _I),
    "tw_vorbis_decode": ([_P, ctypes.c_int64, _P, ctypes.c_int64, _I, ctypes.POINTER(ctypes.c_int64)], _I),
    "tw_vorbis_imdct": ([_P, _I, _P], _I),
    "tw_mp3_probe": ([_P, ctypes.c_int64, ctypes.POINTER(TwMp3Info)], _I),
    "tw_mp3_decode": ([_P, ctypes.c_int64, _P, ctypes.c_int64, _I, ctypes.POINTER(ctypes.c_int64)], _I),
    "tw_aac_parse_asc": ([_P, _I, ctypes.POINTER(TwAacInfo)], _I),
    "tw_aac_decode_raw": ([_P, _I, _P, ctypes.c_int64, _P, _P, ctypes.c_int64, _P, ctypes.c_int64, _I,
                           ctypes.POINTER(ctypes.c_int64)], _I),
    "tw_aac_adts_probe": ([_P, ctypes.c_int64, ctypes.POINTER(TwAacInfo)], _I),
    "tw_aac_adts_decode": ([_P, ctypes.c_int64, _P, ctypes.c_int64, _I, ctypes.POINTER(ctypes.c_int64)], _I),
    "tw_layernorm_set_lds_pad": ([_I], _I),
    "tw_ima_adpcm_wav_decode": ([_P, ctypes.c_int64, _I, _I, _P, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)], _I),
    "tw_ms_adpcm_wav_decode": ([_P, ctypes.c_int64, _I, _I, _P, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)], _I),
    "tw_ima_qt_decode": ([_P, ctypes.c_int64, _I, _P, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)], _I),
    "tw_alac_parse_cookie": ([_P, ctypes.c_int64, _P], _I),
    "tw_alac_decode": ([_P, ctypes.c_int64, _P, ctypes.c_int64, _P, _P, ctypes.c_int64, _P, ctypes.c_int64, _I,
                        ctypes.POINTER(ctypes.c_int64)], _I),
    "tw_resample_pcm_i32": ([_P, ctypes.c_int64, _I, _F, _I, _I, _P, _I, _P, ctypes.c_int64, _P], _I),
    "tw_resample_pcm_f32": ([_P, ctypes.c_int64, _I, _I, _I, _P, _I, _P, ctypes.c_int64, _P], _I),
    "tw_dec_fused": ([_P, _I, _I, _P, _P, _P, _P, _L, _I, _P, _L, _L, _I, _P, _P, _P, _P, _P, _P, _P, _P, _F, _P, _P,
                      _P], _I),
    "tw_dec_fused_xpart_bytes": ([_I], ctypes.c_size_t),
    "tw_dec_fused_sync_bytes": ([], ctypes.c_size_t),
    "tw_dec_fused_supported": ([_I, _I, _I, _I], _I),
    "tw_dec_fused_set_grid": ([_I], _I),
    "tw_dec_fused_set_acquire": ([_I], _I),
    "tw_dec_fused_set_probe": ([_P], _I),
    "tw_dec_fused_grid": ([], _I),
}

_lib = None
_dbg = None


def _open(path: str) -> ctypes.CDLL:
    if not os.path.exists(path):
        raise TwError(f"HIP library not built: {path} (run `make -C turbo-whisper-workspace_amd/csrc`)")
    lib = ctypes.CDLL(path)
    for name, (args, res) in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    return lib


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load (once) and type the library; raises if it is missing. The library is always the in-tree build:
    an environment override (the TW_LIB of old A/B scripts) is refused rather than silently ignored."""
    global _lib
    if _lib is not None:
        return _lib
    if os.environ.get("TW_LIB"):
        raise TwError("TW_LIB is no longer read: A/B builds load their library explicitly (_lib.load_debug or a "
                      "separate process over another in-tree build)")
    _lib = _open(path)
    return _lib


def load_debug() -> ctypes.CDLL:
    """The -DTW_DEBUG=1 build (its own ctypes handle beside the product library; contract checks compiled in)."""
    global _dbg
    if _dbg is None:
        _dbg = _open(DEBUG_LIB_PATH)
        if _dbg.tw_debug_build() != 1:
            raise TwError(f"{DEBUG_LIB_PATH} is not a TW_DEBUG build")
    return _dbg


def call(name: str, *args) -> None:
    """Invoke a tw_* entry point and turn a nonzero return into TwError(tw_last_error())."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        raise TwError(f"{name} failed ({rc}): {lib.tw_last_error().decode(errors='replace')}")


def ptr(t) -> int:
    """Device (or host) address of a torch tensor, or 0 for None."""
    return 0 if t is None else t.data_ptr()


def stream_handle(stream=None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream

"""Token-level timestamps from cross-attention (return_timestamps="word"), host side.

WhisperGenerationMixin._extract_token_timestamps ($TF/models/whisper/generation_whisper.py:241-380) turns the
alignment heads' cross-attention of every fed token into one time per token: crop the frames to num_frames // 2
(generate() passes a per-sample tensor, so the crop is applied twice: :316-323 and :353-354), drop the prompt rows,
standardise every (head, frame) column over the tokens, median-filter each row over frames (width 7, reflect
padding, :43-61), average the heads, dynamic time warping on the negated matrix (tw_dtw in libtwhip.so), and take
the frame of every text-index jump x 0.02 s. The GPU supplies the attention (tw_attn_decode_cross_probs); this
post-processing is O(tokens x frames) host work, as in the reference.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np

from . import _lib


def median_filter(x: np.ndarray, width: int) -> np.ndarray:
    pad = width // 2
    if x.shape[-1] <= pad:
        return x
    xp = np.pad(x, [(0, 0)] * (x.ndim - 1) + [(pad, pad)], mode="reflect")
    return np.sort(np.lib.stride_tricks.sliding_window_view(xp, width, axis=-1), axis=-1)[..., pad]


def dtw(cost: np.ndarray):
    lib = _lib.load()
    cost = np.ascontiguousarray(cost, np.float64)
    n, m = cost.shape
    ti = np.empty(n + m, np.int32)
    tj = np.empty(n + m, np.int32)
    ln = ctypes.c_int32()
    if lib.tw_dtw(cost.ctypes.data, n, m, ti.ctypes.data, tj.ctypes.data, ctypes.byref(ln)) != 0:
        raise _lib.TwError(lib.tw_last_error().decode())
    return ti[: ln.value], tj[: ln.value]


def token_timestamps(weights: np.ndarray, num_input_ids: int, num_frames: Optional[int], median_width: int = 7,
                     time_precision: float = 0.02) -> np.ndarray:
    """weights f32 [heads][rows][frames] of the fed positions (prompt rows first) -> f32 [rows + 1] seconds."""
    rows = weights.shape[1]
    out = np.zeros(rows + 1, np.float32)
    w = np.asarray(weights, np.float32)
    if num_frames is not None:
        w = w[..., : num_frames // 2]
        w = w[..., : num_frames // 2]
    w = w[:, num_input_ids:, :]
    if w.shape[1] == 0:
        return out
    with np.errstate(invalid="ignore", divide="ignore"):
        w = ((w - w.mean(axis=-2, keepdims=True)) / w.std(axis=-2, keepdims=True)).astype(np.float32)
    mat = median_filter(w, median_width).mean(axis=0)
    ti, tj = dtw(-mat.astype(np.float64))
    jumps = np.concatenate([[True], np.diff(ti) != 0])
    jt = tj[jumps] * time_precision
    return np.concatenate([np.zeros(num_input_ids), jt, [jt[-1]]]).astype(np.float32)

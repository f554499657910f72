"""Host-side tables and window arithmetic of the Whisper front end.

* DFT basis / slaney mel filterbank tables consumed by `tw_logmel` (csrc/logmel.hip). The filterbank
  restates `mel_filter_bank(num_frequency_bins=201, num_mel_filters=n_mels, min_frequency=0,
  max_frequency=8000, sampling_rate=16000, norm="slaney", mel_scale="slaney")`
  ($TF/audio_utils.py:448-517, 541-560, 638-729) as WhisperFeatureExtractor.__init__ builds it
  ($TF/models/whisper/feature_extraction_whisper.py:94-102).
* `chunk_windows` restates the ASR pipeline's chunk arithmetic (chunk_iter,
  $TF/pipelines/automatic_speech_recognition.py:61-84, and the sample rounding of preprocess :432-447,
  align_to = 1 for Whisper).
"""
from __future__ import annotations

import math
from typing import Iterator, NamedTuple

import numpy as np

SAMPLE_RATE = 16000
N_FFT = 400
HOP = 160
CHUNK_SAMPLES = 480000  # 30 s, WhisperFeatureExtractor.n_samples
N_FRAMES = 3000
FP = 224  # 201 bins padded to 7 x 32


def _hz_to_mel_slaney(f):
    f = np.asarray(f, dtype=np.float64)
    mels = 3.0 * f / 200.0
    logstep = 27.0 / np.log(6.4)
    return np.where(f >= 1000.0, 15.0 + np.log(np.maximum(f, 1e-300) / 1000.0) * logstep, mels)


def _mel_to_hz_slaney(m):
    m = np.asarray(m, dtype=np.float64)
    freq = 200.0 * m / 3.0
    logstep = np.log(6.4) / 27.0
    return np.where(m >= 15.0, 1000.0 * np.exp(logstep * (m - 15.0)), freq)


def mel_filterbank(n_mels: int, n_freq: int = 201, sr: int = SAMPLE_RATE, fmax: float = 8000.0) -> np.ndarray:
    """Slaney-normalised triangular filters, float64 [n_freq][n_mels]."""
    mel_min, mel_max = _hz_to_mel_slaney(0.0), _hz_to_mel_slaney(fmax)
    mel_pts = np.linspace(mel_min, mel_max, n_mels + 2)
    filt_hz = _mel_to_hz_slaney(mel_pts)
    fft_hz = np.linspace(0, sr // 2, n_freq)
    diff = np.diff(filt_hz)
    slopes = filt_hz[None, :] - fft_hz[:, None]
    down = -slopes[:, :-2] / diff[:-1]
    up = slopes[:, 2:] / diff[1:]
    fb = np.maximum(0.0, np.minimum(down, up))
    enorm = 2.0 / (filt_hz[2 : n_mels + 2] - filt_hz[:n_mels])
    return fb * enorm[None, :]


def dft_basis() -> tuple:
    """Periodic-Hann-windowed DFT basis, f32 [400][224] (cos, -sin); columns >= 201 are zero."""
    n = np.arange(N_FFT, dtype=np.float64)
    w = 0.5 - 0.5 * np.cos(2.0 * np.pi * n / N_FFT)
    f = np.arange(201, dtype=np.float64)
    ang = 2.0 * np.pi * np.outer(n, f) / N_FFT
    c = np.zeros((N_FFT, FP), np.float32)
    s = np.zeros((N_FFT, FP), np.float32)
    c[:, :201] = (w[:, None] * np.cos(ang)).astype(np.float32)
    s[:, :201] = (-w[:, None] * np.sin(ang)).astype(np.float32)
    return c, s


def mel_table(n_mels: int) -> np.ndarray:
    """f32 [224][ceil32(n_mels)] filterbank laid out for tw_logmel (zero padded)."""
    mp = (n_mels + 31) // 32 * 32
    t = np.zeros((FP, mp), np.float32)
    t[:201, :n_mels] = mel_filterbank(n_mels).astype(np.float32)
    return t


def pack_k8(a: np.ndarray) -> np.ndarray:
    """A [K][C] table (K % 8 == 0) in tw_logmel's "k8" order [K/8][C][2][4]: element [k][c] at
    ((k/8 * C + c) * 2 + k%2) * 4 + (k%8)/2, so one 16-byte load holds a column's values for 4 MFMA steps."""
    K, C = a.shape
    assert K % 8 == 0
    return np.ascontiguousarray(a.reshape(K // 8, 4, 2, C).transpose(0, 3, 2, 1))


class Window(NamedTuple):
    start: int       # first sample of the chunk in the input
    length: int      # samples actually present (<= chunk_len)
    stride_left: int
    stride_right: int
    is_last: bool


def chunk_windows(n_samples: int, chunk_length_s: float, stride_length_s=None,
                  sampling_rate: int = SAMPLE_RATE) -> Iterator[Window]:
    """Windows exactly as the ASR pipeline's chunk_iter yields them (samples)."""
    if stride_length_s is None:
        stride_length_s = chunk_length_s / 6
    if isinstance(stride_length_s, (int, float)):
        stride_length_s = [stride_length_s, stride_length_s]
    chunk_len = int(round(chunk_length_s * sampling_rate))
    stride_left = int(round(stride_length_s[0] * sampling_rate))
    stride_right = int(round(stride_length_s[1] * sampling_rate))
    if chunk_len < stride_left + stride_right:
        raise ValueError("Chunk length must be superior to stride length")
    step = chunk_len - stride_left - stride_right
    for start in range(0, n_samples, step):
        end = start + chunk_len
        length = min(end, n_samples) - start
        left = 0 if start == 0 else stride_left
        is_last = end >= n_samples
        right = 0 if is_last else stride_right
        if length > left:
            yield Window(start, length, left, right, is_last)
        if is_last:
            break


def time_precision(max_source_positions: int = 1500) -> float:
    """Seconds per timestamp step (feature_extractor.chunk_length / max_source_positions)."""
    return 30 / max_source_positions


def n_windows_30s(n_samples: int) -> int:
    return max(1, math.ceil(n_samples / CHUNK_SAMPLES))

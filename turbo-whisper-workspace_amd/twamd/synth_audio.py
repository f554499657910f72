"""Seeded synthetic 16 kHz audio for tests and benchmarks (SURVEY.md §8d inputs).

(1) "speech-like": harmonic series at f0 in [90, 250] Hz, 3-6 Hz amplitude modulation, pink noise,
    -20 dBFS; (2) white noise sigma 0.05; (3) silence. numpy PCG64 seeds.
"""
from __future__ import annotations

import numpy as np

SR = 16000


def speech_like(seconds: float, seed: int = 1234) -> np.ndarray:
    rng = np.random.Generator(np.random.PCG64(seed))
    n = int(round(seconds * SR))
    t = np.arange(n) / SR
    f0 = rng.uniform(90, 250)
    # slow pitch drift and syllable-rate amplitude modulation
    f = f0 * (1.0 + 0.05 * np.sin(2 * np.pi * rng.uniform(0.2, 0.5) * t))
    phase = 2 * np.pi * np.cumsum(f) / SR
    x = np.zeros(n)
    for k in range(1, 12):
        x += (1.0 / k) * np.sin(k * phase + rng.uniform(0, 2 * np.pi))
    am = 0.5 * (1.0 + np.sin(2 * np.pi * rng.uniform(3, 6) * t + rng.uniform(0, 2 * np.pi)))
    x *= am
    white = rng.standard_normal(n)
    spec = np.fft.rfft(white)
    fr = np.fft.rfftfreq(n, 1 / SR)
    fr[0] = fr[1] if n > 1 else 1.0
    pink = np.fft.irfft(spec / np.sqrt(fr), n)
    pink /= np.std(pink) + 1e-12
    x = x / (np.sqrt(np.mean(x ** 2)) + 1e-12) + 0.1 * pink
    x *= 0.1 / (np.sqrt(np.mean(x ** 2)) + 1e-12)  # -20 dBFS RMS
    return x.astype(np.float32)


def white_noise(seconds: float, seed: int = 7, sigma: float = 0.05) -> np.ndarray:
    rng = np.random.Generator(np.random.PCG64(seed))
    return (sigma * rng.standard_normal(int(round(seconds * SR)))).astype(np.float32)


def silence(seconds: float) -> np.ndarray:
    return np.zeros(int(round(seconds * SR)), np.float32)


def workload(n_chunks: int, seconds: float = 30.0, seed: int = 1234, zero_frac: float = 0.1) -> np.ndarray:
    """[n_chunks][seconds*SR] batch: speech-like chunks with ~zero_frac silent ones (bench input)."""
    out = np.zeros((n_chunks, int(round(seconds * SR))), np.float32)
    n_zero = int(round(zero_frac * n_chunks))
    for i in range(n_chunks - n_zero):
        out[i] = speech_like(seconds, seed + i)
    return out

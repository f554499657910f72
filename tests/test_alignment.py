"""Token-level timestamps, host side (SURVEY.md §8f "word timestamps"): twamd.alignment (median filter, the
C++ DTW in libtwhip.so, the _extract_token_timestamps post-processing) against the transformers goldens in
tests/golden/word.npz and against the oracle restatement (oracle/whisper_oracle.py) on random inputs."""
import os

import numpy as np
import pytest

from oracle import whisper_oracle as wo
from twamd import alignment

G = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def z():
    return np.load(os.path.join(G, "word.npz"))


def test_native_dtw_matches_transformers(z):
    for k in range(4):
        ti, tj = alignment.dtw(z[f"dtw{k}_in"])
        assert np.array_equal(ti, z[f"dtw{k}_text"]) and np.array_equal(tj, z[f"dtw{k}_time"]), k


@pytest.mark.parametrize("seed", range(6))
def test_native_dtw_matches_oracle_with_ties(seed):
    """Integer-valued costs make every tie rule of the recurrence and the backtrace matter."""
    rng = np.random.default_rng(seed)
    n, m = int(rng.integers(1, 40)), int(rng.integers(1, 120))
    mat = rng.integers(-2, 3, size=(n, m)).astype(np.float64)
    ti, tj = alignment.dtw(mat)
    oi, oj = wo.dynamic_time_warping(mat)
    assert np.array_equal(ti, oi) and np.array_equal(tj, oj)
    assert ti[0] == 0 and tj[0] == 0 and ti[-1] == n - 1 and tj[-1] == m - 1


def test_dtw_rejects_empty():
    with pytest.raises(Exception):
        alignment.dtw(np.zeros((0, 5)))


def test_median_filter_matches_transformers(z):
    np.testing.assert_array_equal(alignment.median_filter(z["median_in"], 7), z["median_out"])
    x = np.arange(3, dtype=np.float32)[None]
    assert np.array_equal(alignment.median_filter(x, 7), x)  # too short to pad: unchanged, as _median_filter


@pytest.mark.parametrize("case", [(4, 3, 20, 1500, 3000), (2, 4, 9, 1500, 1111), (1, 3, 1, 1500, 3000),
                                  (4, 3, 30, 1500, None), (3, 4, 12, 1500, -390), (2, 3, 3, 1500, 2)])
def test_token_timestamps_match_oracle(case):
    heads, P, gen, S, nf = case
    rng = np.random.default_rng(sum(abs(c or 0) for c in case))
    w = rng.random((heads, P + gen, S)).astype(np.float32)
    w /= w.sum(-1, keepdims=True)
    a = alignment.token_timestamps(w, P, nf)
    o = wo.token_timestamps(w, P, nf)
    assert a.dtype == np.float32 and a.shape == (P + gen + 1,)
    np.testing.assert_array_equal(a, o)


def test_token_timestamps_prompt_only():
    w = np.ones((2, 3, 1500), np.float32)
    np.testing.assert_array_equal(alignment.token_timestamps(w, 3, 3000), np.zeros(4, np.float32))

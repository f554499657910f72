"""Check a device decode against the large-v3-turbo goldens (tests/golden/turbo.npz, made by make_golden.py turbo from
transformers on CPU fp32). Test infrastructure: used by tests/test_gpu_turbo.py and by bench.py's parity field; it
reads committed fixtures only (numpy, no oracle, no reference code).

The fp32 sequence is the reference. A bf16 engine may pick the other side of a near-tie; the stated tolerance is
TAU = 0.15 logits on the processed scores (twice the turbo teacher-forced logit tolerance of tests/test_gpu_turbo.py,
itself 3x the measured 0.025): at the
FIRST position where the device token differs, the device token must trail the fp32 choice by at most TAU, or the
timestamp rule (logsumexp of the timestamp log-probs vs the best text log-prob, logits_process.py:2041-2045) must be
within TAU of flipping and the device token be of the other class. After a divergence the prefixes differ and the
fixture has no scores for the device's continuation, so the check stops there."""
from __future__ import annotations

import os
from typing import Dict, Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
TAU = 0.15
BENCH_WINDOWS = (0, 23)  # make_golden.TURBO_BENCH_WINDOWS: bench.py's window 0 (speech) and 23 (silent)
TIMESTAMP_BEGIN = 50365  # large-v3(-turbo) vocabulary


def load(path: str = os.path.join(HERE, "turbo.npz")):
    return np.load(path)


def check_pass(tokens: Sequence[int], gold_tokens: Sequence[int], top_idx: np.ndarray, top_val: np.ndarray,
               ts_margin: np.ndarray, tau: float = TAU, ts_begin: int = TIMESTAMP_BEGIN) -> Dict:
    """Compare one seek pass's generated tokens (prompt excluded, EOS included) with the fp32 pass."""
    tokens = [int(t) for t in tokens]
    gold = [int(t) for t in gold_tokens]
    if tokens == gold:
        return {"status": "exact", "first_divergence": None, "n": len(gold)}
    n = min(len(tokens), len(gold))
    t = next((i for i in range(n) if tokens[i] != gold[i]), n)
    if t >= len(top_idx) or t >= len(tokens):
        return {"status": "mismatch", "first_divergence": t, "n": len(gold), "why": "length"}
    g = tokens[t]
    row_i, row_v = [int(x) for x in top_idx[t]], top_val[t]
    if g in row_i:
        v = float(row_v[row_i.index(g)])
        if np.isfinite(v) and v >= float(row_v[0]) - tau:
            return {"status": "within_tau", "first_divergence": t, "n": len(gold), "gap": float(row_v[0]) - v}
    if abs(float(ts_margin[t])) <= tau and (g >= ts_begin) != (gold[t] >= ts_begin):
        return {"status": "within_tau", "first_divergence": t, "n": len(gold), "rule_margin": float(ts_margin[t])}
    return {"status": "mismatch", "first_divergence": t, "n": len(gold), "device": g, "fp32": gold[t],
            "fp32_top": row_i[:4]}


def check_bench_window(z, w: int, tokens: Sequence[int], lang: int) -> Dict:
    """bench.py's first-pass decode of workload window w (EOS suppressed, 128 new tokens) vs the fp32 golden."""
    r = check_pass(tokens, z[f"bench_w{w}_tokens"], z[f"bench_w{w}_top_idx"], z[f"bench_w{w}_top_val"],
                   z[f"bench_w{w}_ts_margin"])
    r["lang_ok"] = int(lang) == int(z[f"bench_w{w}_lang"][0])
    return r


def gen_passes(z, i: int):
    """The golden generate() passes of clip i: [(seek, tokens, top_idx, top_val, ts_margin), ...]."""
    lens = z[f"gen{i}_pass_len"]
    out, o = [], 0
    for k, n in enumerate(lens):
        out.append((int(z[f"gen{i}_pass_seek"][k]), z[f"gen{i}_pass_tokens"][o: o + n], z[f"gen{i}_top_idx"][o: o + n],
                    z[f"gen{i}_top_val"][o: o + n], z[f"gen{i}_ts_margin"][o: o + n]))
        o += n
    return out

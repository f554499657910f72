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


# ---- every position of the headline workload (turbo_bench.npz, make_golden.py turbo_bench) -------------------------
# The device decode is teacher-forced along each window's fp32 sequence (the captured B = 24 graph the bench times,
# bench.py / tests/test_gpu_turbo.py), so every one of the 128 positions is compared, not only the positions before
# the first divergence. Tolerances: LOGIT_ABS on the fp32 top-16 raw logits and their log-sum-exp (the turbo
# teacher-forced bound of tests/test_gpu_turbo.py, about 3x the measured error); the device's processed argmax is
# the fp32 token or trails it by at most TAU in fp32 processed score; the timestamp-rule margin within TAU of fp32's
# (the rule then decides the same way wherever |fp32 margin| > TAU).
LOGIT_ABS = 0.08
# config 5 (MX-fp8 encoder projections, bf16 decoder): e4m3 operands carry 3 mantissa bits, so the encoder output and
# with it every logit moves by far more than bf16's rounding. Measured at turbo depth (profiles/r03m_fp8_gputest.txt,
# tests/test_gpu_turbo.py): teacher-forced top-16 logits mean |d| 0.16, worst 0.52. Stated bounds, fixed (about 1.5x
# the worst measured): top-16 logits and log-sum-exp within FP8_LOGIT_ABS, the device's processed argmax within
# FP8_TAU of the fp32 choice, the timestamp-rule margin within FP8_TAU, and the mean top-16 error within
# FP8_LOGIT_MEAN_ABS over a window.
FP8_LOGIT_ABS = 0.8
FP8_TAU = 0.8
FP8_LOGIT_MEAN_ABS = 0.3


def load_bench(path: str = os.path.join(HERE, "turbo_bench.npz")):
    return np.load(path)


def ts_rule_margin(s: np.ndarray, tb: int) -> float:
    """logsumexp(timestamp log-probs) - max(text log-probs) of processed scores s (WhisperTimeStampLogitsProcessor,
    $TF/generation/logits_process.py:2041-2045); > 0 masks the text tokens."""
    m = float(np.max(s))
    if not np.isfinite(m):
        return float("-inf")
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        lp = s - (m + np.log(np.sum(np.exp(s - m))))
        ts = lp[tb:]
        mt = np.max(ts)
        lse = mt + np.log(np.sum(np.exp(ts - mt))) if np.isfinite(mt) else -np.inf
        return float(lse - np.max(lp[:tb]))


def process_row(raw: np.ndarray, intervals: np.ndarray, tb: int):
    """The Whisper processor chain on one raw logit row given the history's -inf mask (intervals [lo, hi), from the
    fixture) and the timestamp rule; returns (processed scores f32, rule margin). make_golden.py asserts this equals
    the oracle's process_logits on every fp32 row of the fixture."""
    s = np.asarray(raw, np.float32).copy()
    for lo, hi in np.asarray(intervals).reshape(-1, 2):
        s[lo:hi] = -np.inf
    margin = ts_rule_margin(s, tb)
    if margin > 0:
        s[:tb] = -np.inf
    return s, margin


def check_forced_position(zb, w: int, t: int, raw: np.ndarray, tb: int = TIMESTAMP_BEGIN, logit_abs: float = LOGIT_ABS,
                          tau: float = TAU) -> Dict:
    """Position t of window w: the device's raw logit row when fed the fp32 history, against the fixture."""
    k = f"w{w}_"
    off = zb[k + "mask_off"]
    iv = zb[k + "mask_iv"][off[t]: off[t + 1]]
    raw = np.asarray(raw, np.float32)
    ri, rv = zb[k + "raw_idx"][t], zb[k + "raw_val"][t]
    d_all = np.abs(raw[ri].astype(np.float64) - rv)
    d_top = float(d_all.max())
    mx = float(raw.max())
    lse = mx + float(np.log(np.exp(raw.astype(np.float64) - mx).sum()))
    d_lse = abs(lse - float(zb[k + "lse"][t]))
    s, margin = process_row(raw, iv, tb)
    dev_tok = int(np.argmax(s))
    gold = int(zb[k + "tokens"][t])
    pi, pv = [int(x) for x in zb[k + "top_idx"][t]], zb[k + "top_val"][t]
    if dev_tok == gold:
        gap = 0.0
    elif dev_tok in pi and np.isfinite(pv[pi.index(dev_tok)]):
        gap = float(pv[0]) - float(pv[pi.index(dev_tok)])
    else:
        gap = float("inf")
    fm = float(zb[k + "ts_margin"][t])
    d_margin = 0.0 if fm == margin else abs(margin - fm)  # (equal infinities: the first step masks all text)
    if not np.isfinite(d_margin):
        d_margin = float("inf")
    # a flip of the rule's decision at a near-tie is a class change the token check sees through the margin
    rule_flip_ok = abs(fm) <= tau and (dev_tok >= tb) != (gold >= tb)
    flip = dev_tok != gold and gap > tau and rule_flip_ok
    ok = d_top <= logit_abs and d_lse <= logit_abs and d_margin <= tau and (gap <= tau or flip)
    return {"ok": bool(ok), "d_top": d_top, "d_mean": float(d_all.mean()), "d_lse": d_lse,
            "gap": None if flip else gap, "d_margin": d_margin, "argmax_equal": dev_tok == gold, "rule_flip": bool(flip)}


def summarize_forced(results: Dict[int, list], logit_abs: float = LOGIT_ABS, tau: float = TAU,
                     mean_abs: float = None) -> Dict:
    """{window: [per-position results]} -> bench / test summary (mean_abs: a bound on each window's mean top-16 error)."""
    allr = [r for rs in results.values() for r in rs]
    means = [float(np.mean([r["d_mean"] for r in rs])) for rs in results.values() if rs]
    ok = all(r["ok"] for r in allr) and (mean_abs is None or all(m <= mean_abs for m in means))
    return {"ok": ok, "windows": sorted(int(w) for w in results), "worst_window_mean_d_logit": round(max(means, default=0), 4),
            "positions_checked": len(allr),
            "positions_per_window": sorted({len(rs) for rs in results.values()}),
            "argmax_equal": sum(r["argmax_equal"] for r in allr),
            "worst_d_logit": round(max((r["d_top"] for r in allr), default=0.0), 4),
            "worst_d_lse": round(max((r["d_lse"] for r in allr), default=0.0), 4),
            "worst_d_margin": round(max((r["d_margin"] for r in allr), default=0.0), 4),
            "worst_gap": round(max((r["gap"] for r in allr if r["gap"] is not None), default=0.0), 4),
            "rule_flips": sum(r["rule_flip"] for r in allr),
            "logit_abs": logit_abs, "tau": tau, **({"mean_abs": mean_abs} if mean_abs is not None else {})}


def forced_decode(eng, zb, B: int = 24, T: int = 128, windows=None, fp8: bool = False) -> Dict:
    """Teacher-force every fixture window's fp32 sequence through the engine's captured decode of a B-window batch
    (eng.run_batches([B], max_new_tokens=T, max_passes=1), the call bench.py times: log-mel, encoder, the prompt
    graph with language detection, then the captured fused step, WhisperEngine.step_hook). The waveforms must
    already be in eng.wave[:B] and the EOS-suppressing token list set. windows: a subset of the fixture's windows
    (they must hold the same audio in this batch); fp8: config 5's stated bounds (FP8_*) instead of bf16's. After each step the hook reads the fixture rows' raw logits, checks them
    (check_forced_position) and overwrites those rows' next input with the fp32 token (rows not in the fixture keep
    their own choices). Returns summarize_forced(...) plus the language check."""
    import torch

    wins = [int(w) for w in (zb["windows"] if windows is None else windows)]
    assert max(wins) < B and set(wins) <= {int(w) for w in zb["windows"]}
    la, ta = (FP8_LOGIT_ABS, FP8_TAU) if fp8 else (LOGIT_ABS, TAU)
    res = {w: [] for w in wins}

    def hook(k, v):
        r0, n = (0, B) if v is None else (v.r0, v.n)
        mine = [w for w in wins if r0 <= w < r0 + n]
        if not mine:
            return
        rows = torch.tensor(mine, dtype=torch.int64, device=eng.device)
        lg = eng.logits.index_select(0, rows).cpu().numpy()
        for j, w in enumerate(mine):
            res[w].append(check_forced_position(zb, w, k, lg[j], logit_abs=la, tau=ta))
        if k + 1 < T:
            eng.ids[rows] = torch.tensor([int(zb[f"w{w}_tokens"][k]) for w in mine], dtype=torch.int32,
                                         device=eng.device)
            if v is not None:  # (after the prompt the chains' own priming embeds the forced token)
                eng.embed_head(v)

    eng.step_hook = hook
    try:  # bench.py's own call (one batch: its log-mel + encoder, then the decode pass)
        eng.run_batches([B], task="transcribe", max_new_tokens=T, max_passes=1)
    finally:
        eng.step_hook = None
    out = summarize_forced(res, la, ta, FP8_LOGIT_MEAN_ABS if fp8 else None)
    langs = eng.batch_langs[-1]
    out["lang_ok"] = all(int(langs[w]) == int(zb[f"w{w}_lang"][0]) for w in wins)
    out["ok"] = out["ok"] and out["lang_ok"] and all(len(r) == T for r in res.values())
    out["first_bad"] = next(({"window": w, "position": i, **r} for w in wins for i, r in enumerate(res[w])
                             if not r["ok"]), None)
    return out

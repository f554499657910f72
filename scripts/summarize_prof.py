"""Summarise one gpu_round.sh output directory: the rocprofv3 kernel-trace stats (top kernels by total
time) and the per-kernel HBM traffic from the FETCH_SIZE / WRITE_SIZE PMC passes.

Traffic correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE
reports half the bytes of a wide coalesced streaming read, so read bytes = 2 * FETCH_SIZE * 1024, write
bytes = WRITE_SIZE * 1024.  Writes <dir>/traffic.json {kernel: {"launches", "fetch_kib", "write_kib",
"hbm_bytes"}} (per-launch averages) next to the text summary on stdout.

    python scripts/summarize_prof.py gpurun_out/r01
"""
from __future__ import annotations

import csv
import glob
import json
import os
import sys
from collections import defaultdict


def _find(root: str, pattern: str):
    return sorted(glob.glob(os.path.join(root, "**", pattern), recursive=True))


def kernel_stats(root: str):
    files = _find(os.path.join(root, "kt"), "*kernel_stats.csv")
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]), float(r["AverageNs"]),
                             float(r.get("Percentage", 0.0))))
    rows.sort(key=lambda r: -r[2])
    return rows


def pmc(root: str, sub: str, counter: str):
    per = defaultdict(list)
    for f in _find(os.path.join(root, sub), "*counter_collection.csv"):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r.get("Counter_Name") != counter:
                    continue
                per[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return per


SIMD_NUM = 256 * 4  # MI355X: 256 CUs x 4 SIMDs (rocprofv3's MfmaUtil: busy cycles / (GUI_ACTIVE x SIMD_NUM))
N_XCD = 8  # rocprofv3 sums GRBM_GUI_ACTIVE over the 8 XCDs' GRBMs: one XCD's count is the GPU-active cycles
# (checked: with the sum, k_gemm_8p read 5.3 % busy at 1014 TFLOP/s = 41 % of the MFMA peak; per XCD 42 %)


def mfma_util(root: str):
    """Per kernel (launch-averaged, from the pmc_mfma pass): MFMA busy % of all SIMD cycles while the GPU was active
    (rocprofv3's MfmaUtil formula) and the bf16 MFMA rate from SQ_INSTS_VALU_MFMA_MOPS_BF16 x 512 FLOP over the
    dispatch's own duration (rocprofv3 serialises dispatches under counter collection: each is measured alone)."""
    rows = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(dict)
    for f in _find(os.path.join(root, "pmc_mfma"), "*counter_collection.csv"):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k, d = r["Kernel_Name"], r["Dispatch_Id"]
                rows[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                dur[k][d] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    out = {}
    for k, c in rows.items():
        busy, gui, mops = (sum(c.get(n, [])) for n in ("SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE",
                                                        "SQ_INSTS_VALU_MFMA_MOPS_BF16"))
        ns = sum(dur[k].values())
        if gui > 0 and busy > 0:  # (MX-fp8 kernels count no bf16 MOPS: their busy % is kept, bf16_tflops None)
            out[k] = {"launches": len(dur[k]), "mfma_util_pct": 100.0 * busy / (gui / N_XCD * SIMD_NUM),
                      "bf16_tflops": mops * 512 / ns / 1e3 if ns > 0 and mops > 0 else None}
    return out


def main(root: str) -> None:
    ks = kernel_stats(root)
    print(f"# rocprofv3 --kernel-trace --stats ({root})")
    print(f"{'kernel':70s} {'calls':>6s} {'total_ms':>10s} {'avg_us':>10s} {'pct':>6s}")
    for name, calls, tot, avg, pct in ks[:30]:
        print(f"{name[:70]:70s} {calls:6d} {tot / 1e6:10.3f} {avg / 1e3:10.2f} {pct:6.2f}")
    fetch = pmc(root, "pmc_fetch", "FETCH_SIZE")
    write = pmc(root, "pmc_write", "WRITE_SIZE")
    traffic = {}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [])
        w = write.get(k, [])
        fk = sum(f) / len(f) if f else None
        wk = sum(w) / len(w) if w else None
        hbm = None if fk is None or wk is None else (2.0 * fk + wk) * 1024.0
        traffic[k] = {"launches": max(len(f), len(w)), "fetch_kib": fk, "write_kib": wk, "hbm_bytes": hbm}
    if traffic:
        print("\n# HBM traffic per launch (2*FETCH_SIZE + WRITE_SIZE, KiB -> bytes)")
        for k, v in sorted(traffic.items(), key=lambda kv: -(kv[1]["hbm_bytes"] or 0) * kv[1]["launches"]):
            hb = v["hbm_bytes"]
            print(f"{k[:70]:70s} n={v['launches']:5d} fetch={v['fetch_kib'] or 0:12.0f}KiB "
                  f"write={v['write_kib'] or 0:12.0f}KiB hbm={0 if hb is None else hb / 1e6:10.2f}MB")
    with open(os.path.join(root, "traffic.json"), "w") as fh:
        json.dump(traffic, fh, indent=1)
    mu = mfma_util(root)
    if mu:
        print("\n# MFMA utilisation per launch (pmc_mfma pass: SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs);"
              " bf16 rate = SQ_INSTS_VALU_MFMA_MOPS_BF16 x 512 / dispatch time)")
        for k, v in sorted(mu.items(), key=lambda kv: -kv[1]["mfma_util_pct"]):
            tf = v["bf16_tflops"]
            print(f"{k[:70]:70s} n={v['launches']:5d} mfma_busy={v['mfma_util_pct']:6.1f}% "
                  f"bf16={0 if tf is None else tf:8.1f} TFLOP/s")
        with open(os.path.join(root, "mfma.json"), "w") as fh:
            json.dump(mu, fh, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])

"""Measurement (not a bench line): where the time of one large-M GEMM launch (k_gemm_8p) goes, from per-workgroup
timestamps taken by the kernel itself in the probe build (make -C turbo-whisper-workspace_amd/csrc probe ->
scripts/exp/libtwhip_probe.so, -DTW_GEMM_PROBE). Encoder shapes at M = 36000 (24 windows). Per shape one JSON line:
launch span, per-workgroup prologue / K loop / epilogue medians, the gap between successive workgroups on one CU,
the tail (time with fewer than all CUs busy) and the core clock during the K loop.

    python scripts/exp/gemm_probe.py
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "turbo-whisper-workspace_amd")]
import torch  # noqa: E402

EPI = {"bf16": 0, "gelu_bf16": 1, "resid_f32": 2}  # TW_EPI_* of include/tw_whisper.h (checked below)


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(ROOT, "scripts", "exp", "libtwhip_probe.so"))
    ap.add_argument("--epilogue", type=int, default=0, help="tw_gemm_set_epilogue (1 = transposed accumulators)")
    ap.add_argument("--small", action="store_true", help="only the few-workgroup cases")
    args = ap.parse_args()
    from twamd import _lib
    assert (_lib.TW_EPI_BF16, _lib.TW_EPI_GELU_BF16, _lib.TW_EPI_RESID_F32) == tuple(EPI.values())
    lib = ctypes.CDLL(args.lib)
    lib.tw_gemm_set_epilogue(args.epilogue)
    vp, i = ctypes.c_void_p, ctypes.c_int
    lib.tw_gemm_bf16.argtypes = [vp, vp, i, i, i, i, i, i, vp, i, vp, vp, i, vp, vp]
    lib.tw_gemm_probe_read.argtypes = [vp, i]
    lib.tw_gemm_set_variant(5)
    s = torch.cuda.current_stream().cuda_stream
    # the encoder shapes at 24 windows, then q/k/v at fewer rows: how the epilogue's duration depends on how many
    # workgroups store at once (one round of 15 / 120 / 255 workgroups, then 2 rounds)
    cases = [("qkv", 36000, 3840, 1280, "bf16"), ("o_proj", 36000, 1280, 1280, "resid_f32"),
             ("fc1", 36000, 5120, 1280, "gelu_bf16"), ("fc2", 36000, 1280, 5120, "resid_f32"),
             ("qkv_2K", 36000, 3840, 2560, "bf16")]
    cases += [("qkv_m%d" % m, m, 3840, 1280, "bf16") for m in (256, 2048, 4352, 8704)]
    cases += [("o_proj_m%d" % m, m, 1280, 1280, "resid_f32") for m in (256, 2048, 13056)]
    if args.small:
        cases = [c for c in cases if c[1] < 36000]
    for name, M, N, K, epi in cases:
        A = (torch.randn(M, K, device="cuda") * 0.5).to(torch.bfloat16)
        W = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
        bias = torch.randn(N, device="cuda")
        out = (torch.empty(M, N, dtype=torch.bfloat16, device="cuda") if epi != "resid_f32"
               else torch.zeros(M, N, device="cuda"))
        nwg = -(-M // 256) * -(-N // 256)

        def run():
            rc = lib.tw_gemm_bf16(A.data_ptr(), W.data_ptr(), M, N, K, K, K, EPI[epi], out.data_ptr(), N,
                                  bias.data_ptr(), None, 0, None, s)
            assert rc == 0, rc
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        run()
        e1.record()
        torch.cuda.synchronize()
        ev_us = e0.elapsed_time(e1) * 1e3
        buf = np.zeros(nwg * 16, np.uint64)
        assert lib.tw_gemm_probe_read(buf.ctypes.data, nwg) == 0
        p = buf.reshape(nwg, 16).astype(np.int64)
        t0, t1, t2, t3 = (p[:, k] - p[:, 0].min() for k in range(4))
        us = 0.01  # s_memrealtime ticks at 100 MHz
        span = t3.max() * us
        cu = (p[:, 7] << 16) | ((p[:, 6] >> 8) & 0xFF)  # XCC, then HW_ID's CU / SH / SE fields
        gaps = []
        for c in np.unique(cu):
            idx = np.where(cu == c)[0]
            idx = idx[np.argsort(t0[idx])]
            gaps += list(t0[idx[1:]] - t3[idx[:-1]])
        # busy CUs over time: from start/end events
        ev = np.concatenate([np.stack([t0, np.ones_like(t0)], 1), np.stack([t3, -np.ones_like(t3)], 1)])
        ev = ev[np.argsort(ev[:, 0], kind="stable")]
        busy = np.cumsum(ev[:, 1])
        dt = np.diff(ev[:, 0], append=ev[-1, 0])
        ncu = len(np.unique(cu))
        full = dt[busy >= min(ncu, 256)].sum() * us
        clk = (p[:, 5] - p[:, 4]) / np.maximum(p[:, 2] - p[:, 0], 1) * 100.0  # MHz
        flop = 2.0 * M * N * K
        print(json.dumps({
            "lib": os.path.basename(args.lib), "epilogue": args.epilogue, "shape": name, "M": M, "N": N, "K": K, "epi": epi, "workgroups": nwg, "cus": int(ncu),
            "event_us": round(ev_us, 1), "span_us": round(span, 1), "tflops": round(flop / ev_us / 1e6, 1),
            "prologue_us_med": round(float(np.median(t1 - t0)) * us, 2),
            "kloop_us_med": round(float(np.median(t2 - t1)) * us, 2),
            "kloop_us_p90": round(float(np.percentile(t2 - t1, 90)) * us, 2),
            "epilogue_us_med": round(float(np.median(t3 - t2)) * us, 2),
            "epilogue_us_p90": round(float(np.percentile(t3 - t2, 90)) * us, 2),
            "wg_gap_us_med": round(float(np.median(gaps)) * us if gaps else 0.0, 2),
            "all_cus_busy_us": round(float(full), 1), "tail_us": round(float(span - full), 1),
            "kloop_tflops_per_cu_med": round(2.0 * 256 * 256 * K / float(np.median(t2 - t1) * us) / 1e6, 2),
            "clock_mhz_med": round(float(np.median(clk)), 0),
            # epilogue sub-phases of wave 0 (each after a vmcnt(0)): bias in, half 0 staged, half 0 stored, half 1
            # staged, half 1 stored, then the block's stores retired
            "epi_phases_us_med": [round(float(np.median(p[:, b] - p[:, a])) * us, 2)
                                  for a, b in ((2, 8), (8, 9), (9, 10), (10, 11), (11, 12), (12, 3))],
        }), flush=True)
        del A, W, out


if __name__ == "__main__":
    main()

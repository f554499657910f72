"""Measurement (not a bench line): large-M GEMM kernels against each other (tw_gemm_set_variant: 1 k_gemm_big, 5
k_gemm_8p, 6 k_gemm_8pp) on the encoder shapes at 24 windows (M = 36000, the bench) and 15 windows (M = 22500, one
rank's C3 share), interleaved, median of the per-rep means. One JSON line per case.

    python scripts/gemm_variant_ab.py [--variants 5,6] [--reps 5]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "turbo-whisper-workspace_amd")]
import torch  # noqa: E402

from twamd import _lib  # noqa: E402

NAMES = {1: "k_gemm_big", 5: "k_gemm_8p", 6: "k_gemm_8pp"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="5,6")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--m", default="36000,22500")
    a = ap.parse_args()
    variants = [int(x) for x in a.variants.split(",")]
    _lib.load()
    s = torch.cuda.current_stream().cuda_stream
    E = _lib
    shapes = [("qkv", 3840, 1280, E.TW_EPI_BF16), ("o_proj", 1280, 1280, E.TW_EPI_RESID_F32),
              ("fc1", 5120, 1280, E.TW_EPI_GELU_BF16), ("fc2", 1280, 5120, E.TW_EPI_RESID_F32),
              ("cross_kv", 4 * 2 * 1280, 1280, E.TW_EPI_CROSSKV)]
    for M in (int(x) for x in a.m.split(",")):
        for name, N, K, epi in shapes:
            A = (torch.randn(M, K, device="cuda") * 0.5).to(torch.bfloat16)
            W = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
            bias = torch.randn(N, device="cuda")
            bf = epi in (E.TW_EPI_BF16, E.TW_EPI_GELU_BF16, E.TW_EPI_CROSSKV)
            out = torch.zeros(M * N, dtype=torch.bfloat16 if bf else torch.float32, device="cuda")
            geom = (ctypes.c_int * 4)(1500, M // 1500, 1280, 20) if epi == E.TW_EPI_CROSSKV else None
            flop = 2.0 * M * N * K
            res = {v: [] for v in variants}
            for _ in range(a.reps):
                for v in variants:
                    E.call("tw_gemm_set_variant", v)

                    def run():
                        E.call("tw_gemm_bf16", A.data_ptr(), W.data_ptr(), M, N, K, K, K, epi, out.data_ptr(), N,
                               bias.data_ptr(), None, 0, geom, s)
                    run()
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(a.iters):
                        run()
                    e1.record()
                    torch.cuda.synchronize()
                    res[v].append(e0.elapsed_time(e1) * 1e3 / a.iters)
            med = {v: sorted(x)[len(x) // 2] for v, x in res.items()}
            print(json.dumps({"M": M, "shape": name, "N": N, "K": K,
                              **{NAMES[v] + "_us": round(med[v], 1) for v in variants},
                              **{NAMES[v] + "_tflops": round(flop / med[v] / 1e6, 1) for v in variants}}), flush=True)
            del A, W, out
    E.call("tw_gemm_set_variant", 1)


if __name__ == "__main__":
    main()

"""Measurement (not a bench line): the large-M GEMM kernels with the transposed-accumulator epilogue (tw_gemm_set_epilogue
1) against the f32-image one (0), on the encoder shapes at 24 windows (M = 36000, the bench) and 15 windows (M = 22500,
one rank's C3 share), interleaved (tr 1, 0, 1, 0, ...), median of the per-rep means. One JSON line per case.

    python scripts/gemm_epi_ab.py [--reps 5]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    _lib.load()
    s = torch.cuda.current_stream().cuda_stream
    E = _lib
    shapes = [("qkv", 3840, 1280, E.TW_EPI_BF16), ("o_proj", 1280, 1280, E.TW_EPI_RESID_F32),
              ("fc1", 5120, 1280, E.TW_EPI_GELU_BF16), ("fc2", 1280, 5120, E.TW_EPI_RESID_F32),
              ("cross_kv", 4 * 2 * 1280, 1280, E.TW_EPI_CROSSKV)]
    for M in (36000, 22500):
        for name, N, K, epi in shapes:
            A = (torch.randn(M, K, device="cuda") * 0.5).to(torch.bfloat16)
            W = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
            bias = torch.randn(N, device="cuda")
            bf = epi in (E.TW_EPI_BF16, E.TW_EPI_GELU_BF16, E.TW_EPI_CROSSKV)
            out = torch.zeros(M * N, dtype=torch.bfloat16 if bf else torch.float32, device="cuda")
            geom = (ctypes.c_int * 4)(1500, M // 1500, 1280, 20) if epi == E.TW_EPI_CROSSKV else None
            flop = 2.0 * M * N * K
            for var in (5, 1):
                E.call("tw_gemm_set_variant", var)
                res = {0: [], 1: []}
                for _ in range(a.reps):
                    for tr in (1, 0):
                        E.call("tw_gemm_set_epilogue", tr)

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
                        res[tr].append(e0.elapsed_time(e1) * 1e3 / a.iters)
                med = {tr: sorted(v)[len(v) // 2] for tr, v in res.items()}
                print(json.dumps({"M": M, "shape": name, "N": N, "K": K,
                                  "kernel": "k_gemm_8p" if var == 5 else "k_gemm_big",
                                  "us_tr": round(med[1], 1), "us_f32img": round(med[0], 1),
                                  "tflops_tr": round(flop / med[1] / 1e6, 1), "gain": round(med[0] / med[1], 3)}),
                      flush=True)
            del A, W, out
    E.call("tw_gemm_set_variant", 1)
    E.call("tw_gemm_set_epilogue", 0)


if __name__ == "__main__":
    main()

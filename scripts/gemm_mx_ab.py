"""Measurement (not a bench line): the MX fp8 GEMM kernels (tw_gemm_mx_set_variant 1 k_gemm_mx, 8 k_gemm_8p_mx) on the encoder shapes at 64 windows (M = 96000, BASELINE config 5) and 24 windows, interleaved,
median of the per-rep means. One JSON line per case.

    python scripts/gemm_mx_ab.py [--variants 1,8] [--lib path/to/libtwhip.so]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "turbo-whisper-workspace_amd")]
import torch  # noqa: E402

from twamd import _lib  # noqa: E402

NAMES = {1: "k_gemm_mx", 8: "k_gemm_8p_mx"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="1,8")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--m", default="96000,36000")
    ap.add_argument("--lib", default=None, help="another build of libtwhip.so (A/B across builds)")
    a = ap.parse_args()
    variants = [int(x) for x in a.variants.split(",")]
    _lib.load(a.lib) if a.lib else _lib.load()
    s = torch.cuda.current_stream().cuda_stream
    E = _lib
    shapes = [("qkv", 3840, 1280, E.TW_EPI_BF16), ("o_proj", 1280, 1280, E.TW_EPI_RESID_F32),
              ("fc1", 5120, 1280, E.TW_EPI_GELU_MX), ("fc2", 1280, 5120, E.TW_EPI_RESID_F32)]
    for M in (int(x) for x in a.m.split(",")):
        Mp = (M + 255) // 256 * 256
        for name, N, K, epi in shapes:
            Np = (N + 255) // 256 * 256
            Aq = torch.randint(0, 120, (M, K), dtype=torch.uint8, device="cuda")
            As = torch.full((K // 128, Mp, 4), 127, dtype=torch.uint8, device="cuda")
            Wq = torch.randint(0, 120, (N, K), dtype=torch.uint8, device="cuda")
            Ws = torch.full((K // 128, Np, 4), 120, dtype=torch.uint8, device="cuda")
            bias = torch.randn(N, device="cuda")
            if epi == E.TW_EPI_GELU_MX:
                out = torch.zeros(M, N, dtype=torch.uint8, device="cuda")
                so = torch.zeros(N // 128, Mp, 4, dtype=torch.uint8, device="cuda")
            else:
                out = torch.zeros(M, N, dtype=torch.bfloat16 if epi == E.TW_EPI_BF16 else torch.float32, device="cuda")
                so = None
            flop = 2.0 * M * N * K
            res = {v: [] for v in variants}
            for _ in range(a.reps):
                for v in variants:
                    E.call("tw_gemm_mx_set_variant", v)

                    def run():
                        E.call("tw_gemm_mx", Aq.data_ptr(), As.data_ptr(), Wq.data_ptr(), Ws.data_ptr(), M, N, K, K, K,
                               Mp, Np, epi, out.data_ptr(), N, bias.data_ptr(), None if so is None else so.data_ptr(),
                               Mp if so is not None else 0, s)
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
            del Aq, Wq, out
    E.call("tw_gemm_mx_set_variant", 0)


if __name__ == "__main__":
    main()

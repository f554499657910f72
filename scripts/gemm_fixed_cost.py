"""Measurement (not a bench line): the fixed per-tile cost (prologue + epilogue) of the large-M GEMM kernels, from
launches that differ only in K: t(K) = fixed + K * per_k, so fixed = 2 t(K) - t(2K). Shapes of the encoder (M = 36000
rows, B = 24 windows); bf16 (k_gemm_big / k_gemm_8p) and MX fp8 (k_gemm_mx / k_gemm_8p_mx). One JSON line per case.

    python scripts/gemm_fixed_cost.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "turbo-whisper-workspace_amd")]
import torch  # noqa: E402

from twamd import _lib  # noqa: E402


def timed(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    _lib.load()
    s = torch.cuda.current_stream().cuda_stream
    M = 36000
    for name, N, K, epi in (("qkv", 3840, 1280, _lib.TW_EPI_BF16), ("o_proj", 1280, 1280, _lib.TW_EPI_RESID_F32),
                            ("fc1", 5120, 1280, _lib.TW_EPI_GELU_BF16), ("o_bf16", 1280, 1280, _lib.TW_EPI_BF16)):
        res = {}
        for kk in (K, 2 * K):
            A = (torch.randn(M, kk, device="cuda") * 0.5).to(torch.bfloat16)
            W = (torch.randn(N, kk, device="cuda") * kk ** -0.5).to(torch.bfloat16)
            bias = torch.randn(N, device="cuda")
            out = (torch.empty(M, N, dtype=torch.bfloat16, device="cuda") if epi in (_lib.TW_EPI_BF16, _lib.TW_EPI_GELU_BF16)
                   else torch.zeros(M, N, device="cuda"))
            for var in (1, 5):
                _lib.call("tw_gemm_set_variant", var)
                res[(var, kk)] = timed(lambda: _lib.call("tw_gemm_bf16", A.data_ptr(), W.data_ptr(), M, N, kk, kk, kk,
                                                         epi, out.data_ptr(), N, bias.data_ptr(), None, 0, None, s))
            if epi != _lib.TW_EPI_GELU_BF16:
                Mp, Np = (M + 255) // 256 * 256, (N + 255) // 256 * 256
                Aq = torch.empty(M, kk, dtype=torch.uint8, device="cuda")
                As = torch.zeros(kk // 128, Mp, 4, dtype=torch.uint8, device="cuda")
                Wq = torch.empty(N, kk, dtype=torch.uint8, device="cuda")
                Ws = torch.zeros(kk // 128, Np, 4, dtype=torch.uint8, device="cuda")
                _lib.call("tw_quant_mx", A.data_ptr(), M, kk, kk, Aq.data_ptr(), As.data_ptr(), Mp, s)
                _lib.call("tw_quant_mx", W.data_ptr(), N, kk, kk, Wq.data_ptr(), Ws.data_ptr(), Np, s)
                for mv in (1, 8):
                    _lib.call("tw_gemm_mx_set_variant", mv)
                    res[("mx%d" % mv, kk)] = timed(lambda: _lib.call(
                        "tw_gemm_mx", Aq.data_ptr(), As.data_ptr(), Wq.data_ptr(), Ws.data_ptr(), M, N, kk, kk, kk, Mp,
                        Np, epi, out.data_ptr(), N, bias.data_ptr(), None, 0, s))
                _lib.call("tw_gemm_mx_set_variant", 0)
            del A, W, out
        _lib.call("tw_gemm_set_variant", 1)
        for var in sorted({v for v, _ in res}, key=str):
            t1, t2 = res[(var, K)], res[(var, 2 * K)]
            flop = 2.0 * M * N * K
            print(json.dumps({"shape": name, "kernel": {1: "k_gemm_big", 5: "k_gemm_8p", "mx1": "k_gemm_mx",
                                                        "mx8": "k_gemm_8p_mx"}[var],
                              "us_K": round(t1, 1), "us_2K": round(t2, 1), "fixed_us": round(2 * t1 - t2, 1),
                              "fixed_frac": round((2 * t1 - t2) / t1, 3), "tflops_K": round(flop / t1 / 1e6, 1),
                              "tflops_loop": round(flop / (t2 - t1) / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()

"""A/B timing of the large-M GEMM kernels on the encoder shapes (B=24 windows: M = 36000 rows).
Interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24); random operands.

    python scripts/gemm_bench.py [--rounds 5]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "turbo-whisper-workspace_amd")]
import torch  # noqa: E402

from twamd import _lib  # noqa: E402

SHAPES = [  # name, M, N, K, epi
    ("qkv", 36000, 3840, 1280, _lib.TW_EPI_BF16),
    ("o-proj", 36000, 1280, 1280, _lib.TW_EPI_RESID_F32),
    ("o-bf16", 36000, 1280, 1280, _lib.TW_EPI_BF16),
    ("fc1-bf16", 36000, 5120, 1280, _lib.TW_EPI_BF16),
    ("fc1", 36000, 5120, 1280, _lib.TW_EPI_GELU_BF16),
    ("fc2", 36000, 1280, 5120, _lib.TW_EPI_RESID_F32),
    ("conv2", 36000, 1280, 3840, _lib.TW_EPI_F32),
    ("xkv", 36000, 10240, 1280, _lib.TW_EPI_BF16),
]
if os.environ.get("GEMM_BENCH_B"):  # windows per batch (config 5: 64)
    _M = int(os.environ["GEMM_BENCH_B"]) * 1500
    SHAPES = [(n, _M, N, K, e) for n, _, N, K, e in SHAPES]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    _lib.load()
    s = torch.cuda.current_stream().cuda_stream
    for name, M, N, K, epi in SHAPES:
        A = (torch.randn(M, K, device="cuda") * 0.5).to(torch.bfloat16)
        W = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
        bias = torch.randn(N, device="cuda")
        if epi in (_lib.TW_EPI_BF16, _lib.TW_EPI_GELU_BF16):
            out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        else:
            out = torch.zeros(M, N, device="cuda")
        res = {1: [], 5: [], "blas": [], "mx1": [], "mx8": []}
        mx = name not in ("conv2", "xkv") and not os.environ.get("GEMM_BENCH_NO_MX")  # MX fp8 (config 5) layer shapes
        if mx:
            Mp, Np = (M + 255) // 256 * 256, (N + 255) // 256 * 256
            Aq = torch.empty(M, K, dtype=torch.uint8, device="cuda")
            As = torch.zeros(K // 128, Mp, 4, dtype=torch.uint8, device="cuda")
            Wq = torch.empty(N, K, dtype=torch.uint8, device="cuda")
            Ws = torch.zeros(K // 128, Np, 4, dtype=torch.uint8, device="cuda")
            _lib.call("tw_quant_mx", A.data_ptr(), M, K, K, Aq.data_ptr(), As.data_ptr(), Mp, s)
            _lib.call("tw_quant_mx", W.data_ptr(), N, K, K, Wq.data_ptr(), Ws.data_ptr(), Np, s)
            mepi = _lib.TW_EPI_GELU_MX if epi == _lib.TW_EPI_GELU_BF16 else epi
            if mepi == _lib.TW_EPI_GELU_MX:
                mout = torch.empty(M, N, dtype=torch.uint8, device="cuda")
                mso = torch.zeros(N // 128, Mp, 4, dtype=torch.uint8, device="cuda")
            else:
                mout, mso = out, None
        else:
            del res["mx1"], res["mx8"]
        outs = {}
        for r in range(a.rounds):
            st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            st.record()
            for _ in range(a.iters):  # hipBLASLt through torch (plain GEMM, no fused epilogue) as a yardstick
                torch.nn.functional.linear(A, W)
            en.record()
            torch.cuda.synchronize()
            res["blas"].append(st.elapsed_time(en) / a.iters)
            for v in (1, 5):
                _lib.call("tw_gemm_set_variant", v)
                if epi == _lib.TW_EPI_RESID_F32:
                    out.zero_()
                st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                st.record()
                for _ in range(a.iters):
                    _lib.call("tw_gemm_bf16", A.data_ptr(), W.data_ptr(), M, N, K, K, K, epi, out.data_ptr(), N,
                              bias.data_ptr(), None, 0, None, s)
                en.record()
                torch.cuda.synchronize()
                res[v].append(st.elapsed_time(en) / a.iters)
                if r == 0:
                    outs[v] = out.float().clone() / (a.iters if epi == _lib.TW_EPI_RESID_F32 else 1)
            for mv in ((1, 8) if mx else ()):  # forced kernels (0 = by shape is restored below)
                _lib.call("tw_gemm_mx_set_variant", mv)
                if epi == _lib.TW_EPI_RESID_F32:
                    out.zero_()
                st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                st.record()
                for _ in range(a.iters):
                    _lib.call("tw_gemm_mx", Aq.data_ptr(), As.data_ptr(), Wq.data_ptr(), Ws.data_ptr(), M, N, K, K, K,
                              Mp, Np, mepi, mout.data_ptr(), N, bias.data_ptr(), _lib.ptr(mso), Mp if mso is not None
                              else 0, s)
                en.record()
                torch.cuda.synchronize()
                res[f"mx{mv}"].append(st.elapsed_time(en) / a.iters)
                if r == 0:
                    outs[f"mx{mv}"] = mout.float().clone() / (a.iters if epi == _lib.TW_EPI_RESID_F32 else 1)
        fl = 2.0 * M * N * K
        err = max((outs[1] - outs[v]).abs().max().item() for v in (5,))
        if mx:
            err = max(err, (outs["mx1"] - outs["mx8"]).abs().max().item())
        print(f"{name:7s} M={M} N={N} K={K}: " + "  ".join(
            f"{v}: med {sorted(t)[len(t) // 2]:.3f} ms min {min(t):.3f} ms = {fl / min(t) / 1e9:.0f} TF/s"
            for v, t in res.items()) + f"  max|v1-v5|,|mx1-mx8|={err:.3g}", flush=True)
    _lib.call("tw_gemm_set_variant", 1)
    _lib.call("tw_gemm_mx_set_variant", 0)


if __name__ == "__main__":
    main()

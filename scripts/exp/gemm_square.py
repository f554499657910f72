"""Experiment: large-M GEMM variants on square shapes (calibration against the guide's 8-phase numbers) and hipBLASLt."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "turbo-whisper-workspace_amd")]
import torch  # noqa: E402

from twamd import _lib  # noqa: E402

_lib.load()
s = torch.cuda.current_stream().cuda_stream
for M, N, K in ((4096, 4096, 4096), (8192, 8192, 8192), (36000, 3840, 1280), (36000, 3840, 5120)):
    A = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    W = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    res = {}
    for v in (1, 5, "blas"):
        if v != "blas":
            _lib.call("tw_gemm_set_variant", v)
        best = 1e9
        for _ in range(5):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(5):
                if v == "blas":
                    torch.nn.functional.linear(A, W)
                else:
                    _lib.call("tw_gemm_bf16", A.data_ptr(), W.data_ptr(), M, N, K, K, K, _lib.TW_EPI_BF16,
                              out.data_ptr(), N, None, None, 0, None, s)
            b.record()
            torch.cuda.synchronize()
            best = min(best, a.elapsed_time(b) / 5)
        res[v] = 2.0 * M * N * K / best / 1e9
    print(f"{M}x{N}x{K}: " + "  ".join(f"{k}: {v:.0f} TF/s" for k, v in res.items()), flush=True)
_lib.call("tw_gemm_set_variant", 1)

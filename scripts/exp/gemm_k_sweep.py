"""Experiment: per-tile fixed cost of the large-M GEMM = intercept of time vs K (M=36000, N=3840, bf16 out)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "turbo-whisper-workspace_amd")]
import torch  # noqa: E402

from twamd import _lib  # noqa: E402

_lib.load()
s = torch.cuda.current_stream().cuda_stream
M, N = 36000, 3840
for v in [int(x) for x in (sys.argv[1:] or ["1", "5"])]:
    _lib.call("tw_gemm_set_variant", v)
    for epi, name in ((_lib.TW_EPI_BF16, "bf16"), (_lib.TW_EPI_RESID_F32, "resid")):
        row = []
        for K in (64, 128, 256, 640, 1280, 2560):
            A = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            W = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
            out = torch.zeros(M, N, device="cuda", dtype=torch.bfloat16 if epi == _lib.TW_EPI_BF16 else torch.float32)
            best = 1e9
            for _ in range(5):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(10):
                    _lib.call("tw_gemm_bf16", A.data_ptr(), W.data_ptr(), M, N, K, K, K, epi, out.data_ptr(), N, None,
                              None, 0, None, s)
                b.record()
                torch.cuda.synchronize()
                best = min(best, a.elapsed_time(b) / 10)
            row.append(f"K={K}:{best * 1000:.0f}us")
        print(f"v{v} {name}: " + " ".join(row), flush=True)

"""Experiment: cost of the fused epilogue per GEMM shape (same kernel, epilogue varied), random operands."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "turbo-whisper-workspace_amd")]
import torch  # noqa: E402

from twamd import _lib  # noqa: E402

_lib.load()
s = torch.cuda.current_stream().cuda_stream
for M, N, K in [(36000, 1280, 1280), (36000, 3840, 1280), (36000, 1280, 5120)]:
    A = (torch.randn(M, K, device="cuda") * 0.5).to(torch.bfloat16)
    W = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
    bias = torch.randn(N, device="cuda")
    ob = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    of = torch.zeros(M, N, device="cuda")
    line = []
    for v in (1, 5):
        _lib.call("tw_gemm_set_variant", v)
        for name, epi, out in [("bf16", _lib.TW_EPI_BF16, ob), ("gelu", _lib.TW_EPI_GELU_BF16, ob),
                               ("f32", _lib.TW_EPI_F32, of), ("resid", _lib.TW_EPI_RESID_F32, of)]:
            ts = []
            for r in range(4):
                st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                st.record()
                for _ in range(10):
                    _lib.call("tw_gemm_bf16", A.data_ptr(), W.data_ptr(), M, N, K, K, K, epi, out.data_ptr(), N,
                              bias.data_ptr(), None, 0, None, s)
                en.record()
                torch.cuda.synchronize()
                ts.append(st.elapsed_time(en) / 10)
            line.append(f"v{v}/{name} {min(ts) * 1e3:.0f}us")
    print(f"M={M} N={N} K={K}: " + "  ".join(line), flush=True)
_lib.call("tw_gemm_set_variant", 1)

"""Run one encoder-shape GEMM a few times (for rocprofv3 PMC collection): python scripts/gemm_one.py [shape] [variant]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "turbo-whisper-workspace_amd")]
import torch  # noqa: E402

from twamd import _lib  # noqa: E402

SH = {"qkv": (36000, 3840, 1280, 0), "fc1": (36000, 5120, 1280, 1), "fc2": (36000, 1280, 5120, 2),
      "oproj": (36000, 1280, 1280, 2)}
name = sys.argv[1] if len(sys.argv) > 1 else "qkv"
var = int(sys.argv[2]) if len(sys.argv) > 2 else 1
M, N, K, epi = SH[name]
_lib.load()
_lib.call("tw_gemm_set_variant", var)
A = (torch.randn(M, K, device="cuda") * 0.5).to(torch.bfloat16)
W = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
bias = torch.randn(N, device="cuda")
out = torch.empty(M, N, dtype=torch.bfloat16 if epi < 2 else torch.float32, device="cuda")
for _ in range(4):
    _lib.call("tw_gemm_bf16", A.data_ptr(), W.data_ptr(), M, N, K, K, K, epi, out.data_ptr(), N, bias.data_ptr(), None,
              0, None, torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
print("done")

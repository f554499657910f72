"""Co-residency probe: does a short high-priority kernel (tw_resid_layernorm, 24 rows) start beside a running
k_gemm_big, or wait for GEMM workgroups to retire? Case 'many': a GEMM with ~8 rounds of pending workgroups;
case 'one': a GEMM whose grid fits the chip in one round (256 tiles, long K). Run under rocprofv3 --kernel-trace
and read the small kernels' start times relative to the GEMM (scripts/exp/coresid_report.py)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "turbo-whisper-workspace_amd")]
import torch  # noqa: E402

from twamd import _lib  # noqa: E402

_lib.load()
hi = torch.cuda.Stream(priority=-1)
lo = torch.cuda.Stream(priority=0)
D = 1280
x = torch.randn(24, D, device="cuda")
g = torch.ones(D, device="cuda")
b = torch.zeros(D, device="cuda")
out = torch.empty(24, D, dtype=torch.bfloat16, device="cuda")
cases = {"many": (36000, 5120, 1280), "one": (4096, 4096, 20480)}
bufs = {}
for name, (M, N, K) in cases.items():
    A = (torch.randn(M, K, device="cuda") * 0.1).to(torch.bfloat16)
    W = (torch.randn(N, K, device="cuda") * 0.1).to(torch.bfloat16)
    C = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    bufs[name] = (A, W, C, M, N, K)
torch.cuda.synchronize()
# the same 20 small kernels captured as one graph on the high-priority stream (what the decode step replays)
graph = torch.cuda.CUDAGraph()
hi.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(hi):
    with torch.cuda.graph(graph, stream=hi):
        for i in range(20):
            _lib.call("tw_resid_layernorm", x.data_ptr(), None, 0, None, g.data_ptr(), b.data_ptr(), 24, D, 1e-5,
                      out.data_ptr(), hi.cuda_stream)
torch.cuda.synchronize()
for rep in range(3):
    A, W, C, M, N, K = bufs["many"]
    with torch.cuda.stream(lo):
        _lib.call("tw_gemm_bf16", A.data_ptr(), W.data_ptr(), M, N, K, K, K, _lib.TW_EPI_BF16, C.data_ptr(), N,
                  None, None, 0, None, lo.cuda_stream)
    time.sleep(0.0002)
    with torch.cuda.stream(hi):
        graph.replay()
    torch.cuda.synchronize()
for rep in range(3):
    for name in cases:
        A, W, C, M, N, K = bufs[name]
        with torch.cuda.stream(lo):
            _lib.call("tw_gemm_bf16", A.data_ptr(), W.data_ptr(), M, N, K, K, K, _lib.TW_EPI_BF16, C.data_ptr(), N,
                      None, None, 0, None, lo.cuda_stream)
        time.sleep(0.0002)
        for i in range(20):
            _lib.call("tw_resid_layernorm", x.data_ptr(), None, 0, None, g.data_ptr(), b.data_ptr(), 24, D, 1e-5,
                      out.data_ptr(), hi.cuda_stream)
        torch.cuda.synchronize()
print("done")

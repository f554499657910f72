"""Host cost of hipLaunchKernel on a high-priority stream while another stream has (a) one long kernel queued,
(b) ~100 long kernels queued, (c) ~100 kernels queued each followed by a timing-event pair (what the bench's
encoder prefetch queues)."""
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
M, N, K = 36000, 1280, 1280
A = (torch.randn(M, K, device="cuda") * 0.1).to(torch.bfloat16)
W = (torch.randn(N, K, device="cuda") * 0.1).to(torch.bfloat16)
C = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")


def gemm():
    _lib.call("tw_gemm_bf16", A.data_ptr(), W.data_ptr(), M, N, K, K, K, _lib.TW_EPI_BF16, C.data_ptr(), N, None,
              None, 0, None, lo.cuda_stream)


def small():
    _lib.call("tw_resid_layernorm", x.data_ptr(), None, 0, None, g.data_ptr(), b.data_ptr(), 24, D, 1e-5,
              out.data_ptr(), hi.cuda_stream)


def probe(label, n_queued, events):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n_queued):
        if events:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record(lo)
        gemm()
        if events:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record(lo)
    tq = (time.perf_counter() - t) / max(1, n_queued) * 1e6
    ts = []
    for _ in range(40):
        t = time.perf_counter()
        small()
        ts.append((time.perf_counter() - t) * 1e6)
    torch.cuda.synchronize()
    ts.sort()
    print(f"{label:28s}: queueing {n_queued} GEMMs {tq:7.1f} us each; small launch median {ts[20]:7.1f} us "
          f"max {ts[-1]:7.1f} us", flush=True)


for rep in range(2):
    probe("idle", 0, False)
    probe("one GEMM queued", 1, False)
    probe("100 GEMMs queued", 100, False)
    probe("100 GEMMs + event pairs", 100, True)

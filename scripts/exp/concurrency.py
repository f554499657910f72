"""Experiment: do two hipGraphs replayed on two streams overlap on the GPU? (not product code)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "turbo-whisper-workspace_amd")]
import torch  # noqa: E402

from twamd import _lib  # noqa: E402

_lib.load()
B, D = 12, 1280
dev = "cuda"


def mk(stream, n=100, kind="ln"):
    x = torch.randn(B, D, device=dev)
    parts = torch.randn(4, B, D, device=dev)
    g = torch.ones(D, device=dev)
    hd = torch.empty(B, D, dtype=torch.bfloat16, device=dev)
    W = (torch.randn(5120, D, device=dev) * 0.02).to(torch.bfloat16)
    out = torch.empty(B, 5120, dtype=torch.bfloat16, device=dev)
    bias = torch.zeros(5120, device=dev)

    def f():
        s = stream.cuda_stream
        if kind == "ln":
            _lib.call("tw_resid_layernorm", x.data_ptr(), parts.data_ptr(), 4, g.data_ptr(), g.data_ptr(),
                      g.data_ptr(), B, D, 1e-5, hd.data_ptr(), s)
        else:
            _lib.call("tw_gemm_bf16", hd.data_ptr(), W.data_ptr(), B, 5120, D, D, D, 1, out.data_ptr(), 5120,
                      bias.data_ptr(), None, 0, None, s)
    stream.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(stream):
        f()
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=stream):
            for _ in range(n):
                f()
    torch.cuda.synchronize()
    return gr, (x, parts, g, hd, W, out, bias)


def timeit(pairs, reps=5):
    best = 1e9
    for _ in range(reps):
        torch.cuda.synchronize()
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        for st, gr in pairs:
            st.wait_event(a)
            with torch.cuda.stream(st):
                gr.replay()
        for st, _ in pairs:
            torch.cuda.current_stream().wait_stream(st)
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b))
    return best * 1000 / 100


for kind in ("ln", "gemm"):
    for prio in (0, -1):
        s1 = torch.cuda.Stream(priority=prio)
        s2 = torch.cuda.Stream(priority=prio)
        g1, k1 = mk(s1, kind=kind)
        g2, k2 = mk(s2, kind=kind)
        t1 = timeit([(s1, g1)])
        t2 = timeit([(s2, g2)])
        t12 = timeit([(s1, g1), (s2, g2)])
        print(f"{kind} prio={prio}: A alone {t1:.2f} us/kernel, B alone {t2:.2f}, A||B {t12:.2f} (per kernel-pair)",
              flush=True)

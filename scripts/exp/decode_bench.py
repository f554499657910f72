"""Per-kernel cost of the decoder step at large-v3-turbo dims (B rows), each kernel replayed as a hipGraph of
`n` back-to-back launches (what the captured decode step pays per launch, gaps included).

    python scripts/decode_bench.py [--rows 24] [--n 50]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "turbo-whisper-workspace_amd")]
import torch  # noqa: E402

from twamd import _lib  # noqa: E402


def graph_time(fn, n, reps=5):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn(s.cuda_stream)  # warm
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(n):
                fn(s.cuda_stream)
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b) * 1000 / n)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=24)
    ap.add_argument("--n", type=int, default=50)
    a = ap.parse_args()
    _lib.load()
    B, D, F, H, V, S, T = a.rows, 1280, 5120, 20, 51866, 1500, 448
    dev = "cuda"
    bf = torch.bfloat16

    def rnd(*sh, dt=bf, sc=0.05):
        return (torch.randn(*sh, device=dev) * sc).to(dt)

    x = rnd(B, D, dt=torch.float32, sc=1.0)
    hd = rnd(B, D, sc=1.0)
    ffn = rnd(B, F, sc=1.0)
    Wd = rnd(D, D)
    W1 = rnd(F, D)
    W2 = rnd(D, F)
    Wqkv = rnd(3 * D, D)
    E = rnd(V, D)
    bias = torch.zeros(3 * D, device=dev)
    b1 = torch.zeros(F, device=dev)
    parts = torch.zeros(4, B, D, device=dev)
    out_bf = torch.empty(B, F, dtype=bf, device=dev)
    logits = torch.empty(B, V, device=dev)
    g = torch.ones(D, device=dev)
    bb = torch.zeros(D, device=dev)
    ckv = rnd(2, B, H, S, 64, sc=1.0)
    kc = rnd(B, H, T, 64, sc=1.0)
    vc = rnd(B, H, T, 64, sc=1.0)
    qkvd = rnd(B, 3 * D, sc=1.0)
    att = torch.empty(B, D, dtype=bf, device=dev)
    pos = torch.full((B,), 64, dtype=torch.int32, device=dev)
    ids = torch.zeros(B, dtype=torch.int32, device=dev)
    res = []

    def gemm(A, W, M, N, K, epi, out, bias_t):
        return lambda s: _lib.call("tw_gemm_bf16", A.data_ptr(), W.data_ptr(), M, N, K, K, K, epi, out.data_ptr(), N,
                                   _lib.ptr(bias_t), None, 0, None, s)

    def partial(A, W, M, N, K):
        return lambda s: _lib.call("tw_gemm_bf16_partial", A.data_ptr(), W.data_ptr(), M, N, K, K, K, 4,
                                   parts.data_ptr(), N, s)

    for nw in (0, 4, 8, 16):
        _lib.call("tw_gemm_set_variant", 1 | (nw << 8))
        res.append((f"partial o   N={D} K={D} nw={nw}", graph_time(partial(hd, Wd, B, D, D), a.n), Wd.numel() * 2))
        res.append((f"partial fc2 N={D} K={F} nw={nw}", graph_time(partial(ffn, W2, B, D, F), a.n), W2.numel() * 2))
        res.append((f"fc1 GELU    N={F} K={D} nw={nw}", graph_time(gemm(hd, W1, B, F, D, 1, out_bf, b1), a.n),
                    W1.numel() * 2))
        res.append((f"qkv         N={3 * D} K={D} nw={nw}",
                    graph_time(gemm(hd, Wqkv, B, 3 * D, D, 0, out_bf, bias), a.n), Wqkv.numel() * 2))
        res.append((f"q cross     N={D} K={D} nw={nw}", graph_time(gemm(hd, Wd, B, D, D, 0, out_bf, bias), a.n),
                    Wd.numel() * 2))
        res.append((f"lm head     N={V} K={D} nw={nw}", graph_time(gemm(hd, E, B, V, D, 4, logits, None), a.n),
                    E.numel() * 2))
    _lib.call("tw_gemm_set_variant", 1)
    res.append(("resid_ln 4 parts", graph_time(lambda s: _lib.call(
        "tw_resid_layernorm", x.data_ptr(), parts.data_ptr(), 4, bb.data_ptr(), g.data_ptr(), bb.data_ptr(), B, D,
        1e-5, hd.data_ptr(), s), a.n), 6 * B * D * 4))
    res.append(("attn cross", graph_time(lambda s: _lib.call(
        "tw_attn_decode_cross", hd.data_ptr(), B, H, S, B, None, ckv.data_ptr(), att.data_ptr(), s), a.n),
        ckv.numel() * 2))
    res.append(("attn self t=64", graph_time(lambda s: _lib.call(
        "tw_attn_decode_self", qkvd.data_ptr(), B, H, T, pos.data_ptr(), kc.data_ptr(), vc.data_ptr(), att.data_ptr(),
        s), a.n), 2 * B * H * 65 * 64 * 2))
    res.append(("embed", graph_time(lambda s: _lib.call(
        "tw_embed_decoder", E.data_ptr(), E.data_ptr(), ids.data_ptr(), pos.data_ptr(), B, D, x.data_ptr(), s), a.n),
        B * D * 8))
    from twamd.config import GenerationSettings, PRESETS
    st = GenerationSettings.default(PRESETS["large-v3-turbo"]).special
    p = _lib.TwSelectParams()
    p.V, p.eos, p.pad, p.ts_begin, p.no_timestamps = V, st.eot, st.eot, st.timestamp_begin, st.notimestamps
    p.max_initial_ts, p.use_timestamps, p.max_new, p.mode = 50, 1, 1000000, 0
    state = torch.zeros(B, 8, dtype=torch.int32, device=dev)
    toks = torch.zeros(B, 1 << 20, dtype=torch.int32, device=dev)
    ws = torch.empty(B, _lib.TW_SELECT_WS_PER_ROW, device=dev)
    sup = torch.zeros((V + 31) // 32, dtype=torch.int32, device=dev)
    res.append(("logits select", graph_time(lambda s: _lib.call(
        "tw_logits_select", logits.data_ptr(), B, V, sup.data_ptr(), ctypes.byref(p), state.data_ptr(), None, 448,
        ids.data_ptr(), None, ws.data_ptr(), s), a.n), B * V * 4))
    for name, us, byts in res:
        print(f"{name:34s} {us:8.2f} us  {byts / us / 1e3:8.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()

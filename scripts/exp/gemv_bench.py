"""Per-launch cost of the decoder's packed GEMVs (tw_gemv_packed) and LayerNorms at large-v3-turbo dims, each
replayed as a hipGraph of `n` back-to-back launches (what the captured decode step pays per launch, gaps included),
for every K-slice count the launcher can pick (tw_gemm_set_variant bits 16-23; 0 = its heuristic) and with the
remainder steps batched (default) or one by one (bit 25).

    python scripts/gemv_bench.py [--rows 24] [--n 50] [--kws 0,1,2,4,8]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "turbo-whisper-workspace_amd"), os.path.join(ROOT, "scripts")]
import torch  # noqa: E402

from twamd import _lib  # noqa: E402
from decode_bench import graph_time  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=24)
    ap.add_argument("--n", type=int, default=50)
    ap.add_argument("--kws", default="0,1,2,4,8")
    a = ap.parse_args()
    _lib.load()
    B, D, F, V = a.rows, 1280, 5120, 51866
    dev = "cuda"
    bf = torch.bfloat16

    def rnd(*sh, dt=bf, sc=0.05):
        return (torch.randn(*sh, device=dev) * sc).to(dt)

    def pack(W):
        N, K = W.shape
        Wp = torch.empty((N + 15) // 16 * 16 * K, dtype=bf, device=dev)
        _lib.call("tw_pack_weight", W.data_ptr(), N, K, K, Wp.data_ptr(), torch.cuda.current_stream().cuda_stream)
        return Wp

    Wd, W1, W2, Wqkv, E = (pack(rnd(D, D)), pack(rnd(F, D)), pack(rnd(D, F)), pack(rnd(3 * D, D)), pack(rnd(V, D)))
    hp = rnd(32 * D, sc=1.0)   # packed activations (32-row view)
    fp = rnd(32 * F, sc=1.0)
    att = rnd(B, D, sc=1.0)    # row-major attention output
    parts = torch.zeros(4, B, D, device=dev)
    out_bf = torch.empty(B, 3 * D, dtype=bf, device=dev)
    logits = torch.empty(B, V, device=dev)
    bias = torch.zeros(F, device=dev)
    x = rnd(B, D, dt=torch.float32, sc=1.0)
    g = torch.ones(D, device=dev)
    bb = torch.zeros(D, device=dev)
    torch.cuda.synchronize()
    E_BF16, E_F32, E_GELUP, E_PART = _lib.TW_EPI_BF16, _lib.TW_EPI_F32, _lib.TW_EPI_GELU_PACKED, _lib.TW_EPI_PARTIAL_F32

    def gemv(A, apk, Wp, N, K, epi, out, ldo, bias_t=None, splits=1):
        return lambda s: _lib.call("tw_gemv_packed", A.data_ptr(), apk, K, Wp.data_ptr(), B, N, K, epi, out.data_ptr(),
                                   ldo, _lib.ptr(bias_t), splits, s)

    shapes = [
        ("qkv      N=3840 K=1280", gemv(hp, 1, Wqkv, 3 * D, D, E_BF16, out_bf, 3 * D, bias), 3 * D * D * 2),
        ("o  (att) N=1280 K=1280 s4", gemv(att, 0, Wd, D, D, E_PART, parts, D, None, 4), D * D * 2),
        ("q_x      N=1280 K=1280", gemv(hp, 1, Wd, D, D, E_BF16, out_bf, D, bias), D * D * 2),
        ("fc1 gelu N=5120 K=1280", gemv(hp, 1, W1, F, D, E_GELUP, fp, F, bias), F * D * 2),
        ("fc2      N=1280 K=5120 s4", gemv(fp, 1, W2, D, F, E_PART, parts, D, None, 4), D * F * 2),
        ("proj_out N=51866 K=1280", gemv(hp, 1, E, V, D, E_F32, logits, V), V * D * 2),
    ]
    for serial in (0, 1):
        for kw in [int(k) for k in a.kws.split(",")]:
            _lib.call("tw_gemm_set_variant", 1 | (kw << 16) | (serial << 25))
            for name, fn, byts in shapes:
                us = graph_time(fn, a.n)
                print(f"serial_tail={serial} kw={kw} {name:28s} {us:8.2f} us  {byts / us / 1e3:8.1f} GB/s", flush=True)
    _lib.call("tw_gemm_set_variant", 1)
    # the LayerNorm-fused consumers and the residual-epilogue producers (engine.ln_fused)
    xf = rnd(B, F, dt=torch.float32, sc=1.0)
    gF, bF = torch.ones(F, device=dev), torch.zeros(F, device=dev)

    def gemv_ln(Wp, N, K, epi, out, ldo):
        return lambda s: _lib.call("tw_gemv_packed_ln", x.data_ptr(), g.data_ptr(), bb.data_ptr(), 1e-5, Wp.data_ptr(),
                                   B, N, K, epi, out.data_ptr(), ldo, bias.data_ptr(), s)

    RES = _lib.TW_EPI_RESID_F32
    lst = torch.zeros(D // 16 * 64, device=dev)

    def gemv_lnst(Wp, N, K, epi, out, ldo):
        return lambda s: _lib.call("tw_gemv_packed_lnst", x.data_ptr(), lst.data_ptr(), g.data_ptr(), bb.data_ptr(),
                                   1e-5, Wp.data_ptr(), B, N, K, epi, out.data_ptr(), ldo, bias.data_ptr(), s)

    def gemv_stats(A, apk, Wp, N, K):
        return lambda s: _lib.call("tw_gemv_packed_stats", A.data_ptr(), apk, K, Wp.data_ptr(), B, N, K, x.data_ptr(),
                                   N, bias.data_ptr(), lst.data_ptr(), s)

    fused = [
        ("LNst+q_x N=1280 K=1280", gemv_lnst(Wd, D, D, E_BF16, out_bf, D)),
        ("LNst+fc1 N=5120 K=1280", gemv_lnst(W1, F, D, E_GELUP, fp, F)),
        ("o stats  N=1280 K=1280", gemv_stats(att, 0, Wd, D, D)),
        ("LN+qkv   N=3840 K=1280", gemv_ln(Wqkv, 3 * D, D, E_BF16, out_bf, 3 * D)),
        ("LN+q_x   N=1280 K=1280", gemv_ln(Wd, D, D, E_BF16, out_bf, D)),
        ("LN+fc1   N=5120 K=1280", gemv_ln(W1, F, D, E_GELUP, fp, F)),
        ("o resid  N=1280 K=1280", gemv(att, 0, Wd, D, D, RES, xf, D, bias)),
        ("fc2 resid N=1280 K=5120", gemv(fp, 1, W2, D, F, RES, xf, D, bias)),
    ]
    for kw in [int(k) for k in a.kws.split(",")]:
        _lib.call("tw_gemm_set_variant", 1 | (kw << 16))
        for name, fn in fused:
            print(f"fused kw={kw} {name:28s} {graph_time(fn, a.n):8.2f} us", flush=True)
    _lib.call("tw_gemm_set_variant", 1)
    for nparts in (0, 4):
        us = graph_time(lambda s: _lib.call("tw_resid_layernorm_packed", x.data_ptr(), parts.data_ptr(), nparts,
                                            bb.data_ptr(), g.data_ptr(), bb.data_ptr(), B, D, 1e-5, hp.data_ptr(), s),
                        a.n)
        print(f"resid_ln_packed parts={nparts}             {us:8.2f} us", flush=True)


if __name__ == "__main__":
    main()

"""How much a decoder kernel chain slows down while an encoder GEMM runs beside it (two HIP streams).

Stream E (default priority) runs back-to-back large-M GEMMs of an encoder shape; stream D (high priority) replays a
hipGraph of n back-to-back launches of one decoder kernel. Per decoder kernel kind: microseconds per launch with D
alone, and while E is busy (D's graph replayed repeatedly inside E's window). A fixed per-launch penalty in the
concurrent column means kernel boundaries cost; a proportional one means bandwidth / issue sharing.

    python scripts/exp/interference.py [--variant 1] [--epi 2] [--n 40]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "turbo-whisper-workspace_amd")]
import torch  # noqa: E402

from twamd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", type=int, default=1)  # encoder GEMM kernel (tw_gemm_set_variant)
    ap.add_argument("--epi", type=int, default=2)      # 2 = RESID_F32 (o-proj / fc2), 1 = GELU_BF16 (fc1)
    ap.add_argument("--n", type=int, default=40)
    ap.add_argument("--gemms", type=int, default=60)
    ap.add_argument("--attn-pad", type=int, default=0)  # encoder attention LDS padding, 16 KiB units
    ap.add_argument("--kw", type=int, default=0)  # force the packed GEMV's K-slices per column group (0: heuristic)
    a = ap.parse_args()
    _lib.load()
    dev = "cuda"
    bf = torch.bfloat16
    B, D, F, H, S, V = 24, 1280, 5120, 20, 1500, 51866
    M = B * S

    def rnd(*sh, dt=bf, sc=0.05):
        return (torch.randn(*sh, device=dev) * sc).to(dt)

    # encoder operands
    N, K = (D, F) if a.epi == 2 else (F, D)
    A = rnd(M, K, sc=1.0)
    W = rnd(N, K)
    bias = torch.zeros(N, device=dev)
    out = torch.zeros(M, N, dtype=torch.float32 if a.epi == 2 else bf, device=dev)

    # decoder operands
    def pack(Wt):
        n, k = Wt.shape
        Wp = torch.empty((n + 15) // 16 * 16 * k, dtype=bf, device=dev)
        _lib.call("tw_pack_weight", Wt.data_ptr(), n, k, k, Wp.data_ptr(), torch.cuda.current_stream().cuda_stream)
        return Wp

    Wqkv, Wd, Wlm = pack(rnd(3 * D, D)), pack(rnd(D, D)), pack(rnd(V, D))
    hp = rnd(32 * D, sc=1.0)
    qkv = torch.empty(B, 3 * D, dtype=bf, device=dev)
    parts = torch.zeros(4, B, D, device=dev)
    att = rnd(B, D, sc=1.0)
    logits = torch.empty(B, V, device=dev)
    x = rnd(B, D, dt=torch.float32, sc=1.0)
    g = torch.ones(D, device=dev)
    bb = torch.zeros(D, device=dev)
    ckv = rnd(2, B, H, S, 64, sc=1.0)
    q = rnd(B, D, sc=1.0)
    ids = torch.zeros(B, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()

    kinds = {
        "gemv qkv (240 WGs)": lambda s: _lib.call("tw_gemv_packed", hp.data_ptr(), 1, D, Wqkv.data_ptr(), B, 3 * D, D,
                                                  _lib.TW_EPI_BF16, qkv.data_ptr(), 3 * D, None, 1, s),
        "gemv o split4": lambda s: _lib.call("tw_gemv_packed", att.data_ptr(), 0, D, Wd.data_ptr(), B, D, D,
                                             _lib.TW_EPI_PARTIAL_F32, parts.data_ptr(), D, None, 4, s),
        "resid_ln (24 WGs)": lambda s: _lib.call("tw_resid_layernorm_packed", x.data_ptr(), parts.data_ptr(), 4,
                                                 bb.data_ptr(), g.data_ptr(), bb.data_ptr(), B, D, 1e-5, hp.data_ptr(),
                                                 s),
        "cross attn (480 WGs)": lambda s: _lib.call("tw_attn_decode_cross", q.data_ptr(), B, H, S, B, None,
                                                    ckv.data_ptr(), att.data_ptr(), s),
        "proj_out gemv": lambda s: _lib.call("tw_gemv_packed", hp.data_ptr(), 1, D, Wlm.data_ptr(), B, V, D,
                                             _lib.TW_EPI_F32, logits.data_ptr(), V, None, 1, s),
        "embed (24 tiny WGs)": lambda s: _lib.call("tw_embed_decoder", att.data_ptr(), att.data_ptr(), ids.data_ptr(),
                                                   ids.data_ptr(), B, D, x.data_ptr(), s),
    }
    sE = torch.cuda.Stream(priority=0)
    sD = torch.cuda.Stream(priority=-1)
    _lib.call("tw_gemm_set_variant", (a.variant if a.variant < 100 else 1) | (a.kw << 16))
    _lib.call("tw_attn_set_variant", 16); _lib.call("tw_attn_set_lds_pad", a.attn_pad)

    nb = None
    if a.variant in (103, 104):
        import ctypes
        nb = ctypes.CDLL(os.path.join(ROOT, "scripts", "exp", "libneighbors.so"))
    nbout = torch.zeros(4096, device=dev)
    qkv_enc = rnd(M, 3 * D, sc=1.0)
    att_enc = torch.empty(M, D, dtype=bf, device=dev)
    xe = torch.randn(M, D, device=dev)
    hln = torch.empty(M, D, dtype=bf, device=dev)
    Wt = W.t()

    def enc(n):
        for _ in range(n):
            if a.variant == 100:  # hipBLASLt as a yardstick (plain GEMM, no fused epilogue)
                torch.matmul(A, Wt, out=out) if out.dtype == bf else torch.matmul(A, Wt)
            elif a.variant == 101:  # encoder self-attention
                _lib.call("tw_attn_encoder", qkv_enc.data_ptr(), B, S, H, att_enc.data_ptr(), sE.cuda_stream)
            elif a.variant == 102:  # encoder LayerNorm
                _lib.call("tw_layernorm", xe.data_ptr(), g.data_ptr(), bb.data_ptr(), M, D, 1e-5, hln.data_ptr(),
                          sE.cuda_stream)
            elif a.variant == 103:  # synthetic: MFMAs only, one 136 KiB workgroup per CU (scripts/exp/neighbors.hip)
                nb.nb_mfma_spin(ctypes.c_void_p(nbout.data_ptr()), 2048, 20000, ctypes.c_void_p(sE.cuda_stream))
            elif a.variant == 104:  # synthetic: LDS-DMA HBM streaming only, same occupancy
                nb.nb_mem_stream(ctypes.c_void_p(A.data_ptr()), ctypes.c_size_t(A.numel() * 2),
                                 ctypes.c_void_p(nbout.data_ptr()), 2048, 64, ctypes.c_void_p(sE.cuda_stream))
            else:
                _lib.call("tw_gemm_bf16", A.data_ptr(), W.data_ptr(), M, N, K, K, K, a.epi, out.data_ptr(), N,
                          bias.data_ptr(), None, 0, None, sE.cuda_stream)

    # encoder alone
    with torch.cuda.stream(sE):
        enc(2)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(sE)
        enc(a.gemms)
        e1.record(sE)
    torch.cuda.synchronize()
    t_enc = e0.elapsed_time(e1) / a.gemms
    flop = 2.0 * M * N * K
    print(f"encoder GEMM variant {a.variant} epi {a.epi} M={M} N={N} K={K}: {t_enc * 1e3:.1f} us/launch "
          f"({flop / t_enc / 1e9:.0f} TF/s alone)", flush=True)
    for name, fn in kinds.items():
        g_ = torch.cuda.CUDAGraph()
        sD.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(sD):
            fn(sD.cuda_stream)
            torch.cuda.synchronize()
            with torch.cuda.graph(g_, stream=sD):
                for _ in range(a.n):
                    fn(sD.cuda_stream)
        torch.cuda.synchronize()
        # alone
        best = 1e9
        for _ in range(5):
            d0, d1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            d0.record(sD)
            with torch.cuda.stream(sD):
                g_.replay()
            d1.record(sD)
            torch.cuda.synchronize()
            best = min(best, d0.elapsed_time(d1))
        alone = best * 1e3 / a.n
        # beside the encoder: queue the GEMMs, then replay D's graph while they run
        with torch.cuda.stream(sE):
            enc(a.gemms)
            eend = torch.cuda.Event()
            eend.record(sE)
        times = []
        for _ in range(200):
            d0, d1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            d0.record(sD)
            with torch.cuda.stream(sD):
                g_.replay()
            d1.record(sD)
            d1.synchronize()
            if eend.query():
                break
            times.append(d0.elapsed_time(d1) * 1e3 / a.n)
        torch.cuda.synchronize()
        times.sort()
        med = times[len(times) // 2] if times else float("nan")
        print(f"{name:24s} alone {alone:7.2f} us/launch   beside encoder median {med:7.2f} us/launch "
              f"(n={len(times)} replays)", flush=True)
    # encoder slowdown with a decode-like chain beside it
    fn = kinds["gemv qkv (240 WGs)"]
    g_ = torch.cuda.CUDAGraph()
    with torch.cuda.stream(sD):
        with torch.cuda.graph(g_, stream=sD):
            for _ in range(a.n):
                fn(sD.cuda_stream)
    torch.cuda.synchronize()
    with torch.cuda.stream(sE):
        e0.record(sE)
        enc(a.gemms)
        e1.record(sE)
    while not e1.query():
        with torch.cuda.stream(sD):
            g_.replay()
        torch.cuda.current_stream().wait_stream(sD)
        sD.synchronize()
    torch.cuda.synchronize()
    t2 = e0.elapsed_time(e1) / a.gemms
    print(f"encoder GEMM beside a gemv chain: {t2 * 1e3:.1f} us/launch ({flop / t2 / 1e9:.0f} TF/s)", flush=True)


if __name__ == "__main__":
    main()

"""Measurement (not a bench line): per-launch cost of single decoder-step kernels in a captured chain of identical
launches (warm caches, same inputs every launch), at large-v3-turbo dims and R rows, beside a chain of trivial
kernels. Pairs "X + trivial" show what a kernel costs behind a light predecessor. One JSON line per case.

    python scripts/decode_kernel_chains.py [--rows 24] [--n 32] [--reps 20]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "turbo-whisper-workspace_amd")]
import torch  # noqa: E402

from twamd import _lib  # noqa: E402
from twamd.config import PRESETS, GenerationSettings  # noqa: E402
from twamd.engine import LN_EPS, WhisperEngine  # noqa: E402
from twamd.synth_audio import workload  # noqa: E402
from twamd.weights import build_weights  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=24)
    ap.add_argument("--n", type=int, default=32)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--pos", type=int, default=64)
    ap.add_argument("--flush", type=int, default=0)
    a = ap.parse_args()
    dims = PRESETS["large-v3-turbo"]
    gen = GenerationSettings.default(dims)
    R = a.rows
    eng = WhisperEngine(build_weights(dims, seed=1234), gen, max_batch=R, device="cuda")
    eng.wave[:R].copy_(torch.from_numpy(workload(R, 30.0, seed=1234)))
    eng.logmel(R)
    eng.row_map[:R] = torch.arange(R, dtype=torch.int32)
    eng.seek[:R] = 0
    eng.encode(R)
    torch.cuda.synchronize()
    v = eng._view(0, R)
    D, F, H, T = dims.d_model, dims.ffn, dims.heads, dims.max_target_positions
    L = eng.w.dec[0]
    P = eng.dec_p[0]
    s = eng.stream.cuda_stream
    eng.pos[:R] = a.pos
    eng.ids[:R] = 50300
    x_out = torch.empty_like(eng.xd)
    tiny = torch.zeros(64, device="cuda")

    def trivial():
        tiny.add_(1.0)

    def resid_ln4():
        _lib.call("tw_resid_layernorm_packed_to", v.xd.data_ptr(), x_out.data_ptr(), v.parts.data_ptr(), 4,
                  L.bo.data_ptr(), L.ln2_g.data_ptr(), L.ln2_b.data_ptr(), R, D, LN_EPS, v.hp.data_ptr(), s)

    def ln_only():
        _lib.call("tw_resid_layernorm_packed_to", v.xd.data_ptr(), x_out.data_ptr(), None, 0, None,
                  L.ln2_g.data_ptr(), L.ln2_b.data_ptr(), R, D, LN_EPS, v.hp.data_ptr(), s)

    def gemv(key, N, K, epi, out, a_src, packed, splits=1, bias=None):
        def f():
            eng._gemv(a_src, packed, P[key], R, N, K, epi, out, v, bias=bias, splits=splits)
        return f

    BF, PART, GP = _lib.TW_EPI_BF16, _lib.TW_EPI_PARTIAL_F32, _lib.TW_EPI_GELU_PACKED
    kc, vc = eng.kcache[0].data_ptr(), eng.vcache[0].data_ptr()

    def self_attn():
        _lib.call("tw_attn_decode_self", v.qkvd.data_ptr(), R, H, T, v.pos.data_ptr(), kc, vc, v.attd.data_ptr(), s)

    xkv_stride = 2 * R * H * 1500 * 64
    ckv, rmap = eng._cross_ptrs(0, xkv_stride, v)

    def cross_attn():
        _lib.call("tw_attn_decode_cross", v.qd.data_ptr(), R, H, 1500, R, rmap, ckv, v.attd.data_ptr(), s)

    def proj_out():
        eng._gemv(v.hp, True, eng.emb_p, R, dims.vocab, D, _lib.TW_EPI_F32, v.logits, v)

    cases = [
        ("trivial", trivial), ("resid_ln4", resid_ln4), ("ln_only", ln_only),
        ("qkv", gemv("wqkv", 3 * D, D, BF, v.qkvd, v.hp, True, bias=L.bqkv)),
        ("o_proj", gemv("wo", D, D, PART, v.parts, v.attd, False, splits=4)),
        ("q_x", gemv("wq_x", D, D, BF, v.qd, v.hp, True, bias=L.bq_x)),
        ("fc1", gemv("w1", F, D, GP, v.fp, v.hp, True, bias=L.b1)),
        ("fc2", gemv("w2", D, F, PART, v.parts, v.fp, True, splits=4)),
        ("self_attn", self_attn), ("cross_attn", cross_attn), ("proj_out", proj_out),
    ]

    def timed(fn, n):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(eng.stream):
            fn()
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=eng.stream):
                for _ in range(n):
                    fn()
            for _ in range(3):
                g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(eng.stream)
            for _ in range(a.reps):
                g.replay()
            e1.record(eng.stream)
            torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / a.reps / n

    t_triv = timed(trivial, a.n)
    if a.flush:
        # where a cold GEMV's weights come from: X behind a copy that evicts the L2s only (2 x 20 MB moved) or the
        # Infinity Cache too (2 x 300 MB), against X behind a trivial kernel (everything warm)
        for mb in (20, 300):
            src = torch.empty(mb << 18, device="cuda")  # mb MiB of f32
            dst = torch.empty_like(src)

            def flush(src=src, dst=dst):
                dst.copy_(src)
            t_f = timed(flush, a.n // 2)
            for name, fn in cases:
                if name not in ("qkv", "fc1", "q_x", "o_proj", "resid_ln4"):
                    continue

                def pair(fn=fn, flush=flush):
                    fn()
                    flush()
                tp = timed(pair, a.n // 2) - t_f
                print(json.dumps({"rows": R, "kernel": name, "behind_copy_MiB": mb, "us": round(tp, 2),
                                  "copy_alone_us": round(t_f, 2)}), flush=True)
        return
    for var in (0, 1):
        _lib.call("tw_gemv_set_variant", var)
        for name, fn in cases:
            if var == 1 and name not in ("qkv", "o_proj", "q_x", "fc1", "fc2"):
                continue
            t = timed(fn, a.n)

            def pair(fn=fn):
                fn()
                trivial()
            tp = timed(pair, a.n // 2) - t_triv
            print(json.dumps({"rows": R, "gemv_variant": var, "kernel": name, "chain_us": round(t, 2),
                              "behind_trivial_us": round(tp, 2)}), flush=True)
    _lib.call("tw_gemv_set_variant", 0)


if __name__ == "__main__":
    main()

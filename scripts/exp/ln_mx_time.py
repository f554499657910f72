"""Measurement (not a bench line): tw_layernorm_mx (f32 rows -> MX fp8 + scales) at the encoder shapes, M = 96000 and
36000 rows of D = 1280, per launch (median of reps x iters), with the algorithmic bytes (f32 row in, fp8 row + scale
bytes out) as GB/s; optionally from another build (--lib). Outputs are hashed so two builds can be compared bit for bit.

    python scripts/exp/ln_mx_time.py [--lib path/to/libtwhip.so]
"""
import argparse
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "turbo-whisper-workspace_amd")]
import torch  # noqa: E402

from twamd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    _lib.load(a.lib) if a.lib else _lib.load()
    s = torch.cuda.current_stream().cuda_stream
    D = 1280
    g = torch.Generator(device="cuda").manual_seed(7)
    gam = torch.randn(D, device="cuda", generator=g) * 0.2 + 1.0
    bet = torch.randn(D, device="cuda", generator=g) * 0.1
    for M in (96000, 36000):
        x = torch.randn(M, D, device="cuda", generator=g) * 3.0
        q = torch.empty(M, D, dtype=torch.uint8, device="cuda")
        sc = torch.zeros(D // 128, M, 4, dtype=torch.uint8, device="cuda")

        def run():
            _lib.call("tw_layernorm_mx", x.data_ptr(), gam.data_ptr(), bet.data_ptr(), M, D, 1e-5, q.data_ptr(),
                      sc.data_ptr(), M, s)
        run()
        torch.cuda.synchronize()
        digest = hashlib.sha256(q.cpu().numpy().tobytes() + sc.cpu().numpy().tobytes()).hexdigest()[:16]
        ts = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                run()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3 / a.iters)
        us = sorted(ts)[len(ts) // 2]
        nbytes = M * D * 4 + M * D + M * D // 32
        print(json.dumps({"M": M, "D": D, "us": round(us, 1), "GB/s": round(nbytes / us / 1e3, 1), "out_sha": digest}),
              flush=True)


if __name__ == "__main__":
    main()

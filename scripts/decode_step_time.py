"""Measurement (not a bench line): the greedy decode pass alone (no encoder beside it) at large-v3-turbo dims, per
decoder step (47 launches per token), for several row counts. One pass = the prompt graph (SOT, language
detection, task token) + 128 generated tokens with EOS suppressed, i.e. 130 decoder steps; the encoder runs once
before, untimed. Prints one JSON line per (rows, mode).

    python scripts/decode_step_time.py [--rows 15 24 64] [--reps 3] [--fused 0 1]

--fused 1: the decoder's layers as one persistent launch (tw_dec_fused) at every row count <= 32, 0: the launch chain
(WhisperEngine.dec_fused_alone / dec_fused_max_rows overridden); with both, each row count runs both and reports
whether their tokens agree.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "turbo-whisper-workspace_amd")]
import torch  # noqa: E402

from twamd.config import PRESETS, GenerationSettings  # noqa: E402
from twamd.engine import WhisperEngine  # noqa: E402
from twamd.synth_audio import workload  # noqa: E402
from twamd.weights import build_weights  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, nargs="+", default=[15, 24, 64])
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--check-every", type=int, nargs="+", default=[8])
    ap.add_argument("--graph-steps", type=int, nargs="+", default=[1])
    ap.add_argument("--fused", type=int, nargs="+", default=[0])
    ap.add_argument("--slope", type=int, default=0, help="also time 64-token passes: per-step slope without the "
                    "pass's fixed costs")
    a = ap.parse_args()
    dims = PRESETS["large-v3-turbo"]
    gen = GenerationSettings.default(dims)
    B = max(a.rows)
    eng = WhisperEngine(build_weights(dims, seed=1234), gen, max_batch=B, device="cuda")
    eng.set_suppress_tokens(list(gen.suppress_tokens) + [gen.special.eot])
    eng.wave[:B].copy_(torch.from_numpy(workload(B, 30.0, seed=1234)))
    eng.logmel(B)
    tail = eng.prompt_tail("transcribe", True)
    for R in a.rows:
        eng.row_map[:R] = torch.arange(R, dtype=torch.int32)
        eng.seek[:R] = 0
        eng.encode(R)
        torch.cuda.synchronize()
        ref = None
        for fz, ce, gs in [(f, c, g) for f in a.fused for c in a.check_every for g in a.graph_steps]:
            if fz and R > 32:
                continue
            eng.dec_fused_alone = bool(fz)
            eng.dec_fused_max_rows = 32 if fz else 0
            eng.graph_steps_alone = gs
            eng._graphs.clear()
            eng.decode_pass(R, tail, None, 128, check_every=ce)  # warm-up: graph captures
            torch.cuda.synchronize()
            best = 1e9
            eng.pass_events = []
            for _ in range(a.reps):
                t0 = time.perf_counter()
                res = eng.decode_pass(R, tail, None, 128, check_every=ce)
                torch.cuda.synchronize()
                best = min(best, time.perf_counter() - t0)
            loop_us = min(e0.elapsed_time(e1) * 1e3 / n for e0, e1, n, _ in eng.pass_events)
            eng.pass_events = None
            print(json.dumps({"rows": R, "fused": fz, "check_every": ce, "graph_steps": gs,
                              "loop_us_per_step": round(loop_us, 1)}),
                  flush=True)
            assert all(len(t) == 128 for t in res.tokens)
            ref = res.tokens if ref is None else ref
            if a.slope:
                eng.decode_pass(R, tail, None, 64, check_every=ce)
                torch.cuda.synchronize()
                b64 = 1e9
                for _ in range(a.reps):
                    t0 = time.perf_counter()
                    eng.decode_pass(R, tail, None, 64, check_every=ce)
                    torch.cuda.synchronize()
                    b64 = min(b64, time.perf_counter() - t0)
                print(json.dumps({"rows": R, "check_every": ce, "graph_steps": gs,
                                  "pass64_ms": round(b64 * 1e3, 2),
                                  "slope_us_per_step": round((best - b64) * 1e6 / 64, 1),
                                  "fixed_ms": round((b64 - 66 * (best - b64) / 64) * 1e3, 2)}), flush=True)
            print(json.dumps({"rows": R, "fused": fz, "check_every": ce, "graph_steps": gs,
                              "pass_ms": round(best * 1e3, 2),
                              "step_us": round(best * 1e6 / 130, 1), "tokens_equal": res.tokens == ref}),
                  flush=True)


if __name__ == "__main__":
    main()

"""Measurement (not a bench line): the greedy decode pass alone (no encoder beside it) at large-v3-turbo dims, per
decoder step (47 launches per token), for several row counts. One pass = the prompt graph (SOT, language
detection, task token) + 128 generated tokens with EOS suppressed, i.e. 130 decoder steps; the encoder runs once
before, untimed. Prints one JSON line per (rows, mode).

    python scripts/decode_step_time.py [--rows 15 24 64] [--reps 3]
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
        for mode in ("separate",):
            eng._graphs.clear()
            eng.decode_pass(R, tail, None, 128)  # warm-up: graph captures
            torch.cuda.synchronize()
            best = 1e9
            for _ in range(a.reps):
                t0 = time.perf_counter()
                res = eng.decode_pass(R, tail, None, 128)
                torch.cuda.synchronize()
                best = min(best, time.perf_counter() - t0)
            assert all(len(t) == 128 for t in res.tokens)
            print(json.dumps({"rows": R, "mode": mode, "pass_ms": round(best * 1e3, 2),
                              "step_us": round(best * 1e6 / 130, 1)}), flush=True)


if __name__ == "__main__":
    main()

"""Interleaved A/B of the large-M GEMM kernel queued beside a running decode (tw_gemm_set_variant: 1 = k_gemm_big,
the default, 5 = k_gemm_8p) in the bench workload (config 2: 24 windows, 128 tokens, overlapped pipeline), one
process. Re-measures round 2's finding with the round-3 decoder kernels.   python scripts/exp/ab_gemm_beside.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "turbo-whisper-workspace_amd")]
import torch  # noqa: E402

from twamd import _lib  # noqa: E402
from twamd.config import PRESETS, GenerationSettings  # noqa: E402
from twamd.engine import WhisperEngine  # noqa: E402
from twamd.synth_audio import workload  # noqa: E402
from twamd.weights import build_weights  # noqa: E402

steps, rounds = 8, 3
dims = PRESETS["large-v3-turbo"]
gen = GenerationSettings.default(dims)
eng = WhisperEngine(build_weights(dims, seed=1234), gen, max_batch=24, device="cuda:0")
eng.set_suppress_tokens(list(gen.suppress_tokens) + [gen.special.eot])
eng.wave[:24].copy_(torch.from_numpy(workload(24, 30.0, seed=1234)))
orig = eng._set_gemm_context


def ctx_for(beside):
    def f(alone):
        orig(alone)
        if not alone:
            _lib.call("tw_gemm_set_variant", beside)
    return f


res, toks = {1: [], 5: []}, {}
for r in range(rounds):
    for beside in (1, 5):
        eng._set_gemm_context = ctx_for(beside)
        eng.run_batches([24] * 2, task="transcribe", max_new_tokens=128, max_passes=1)  # warm (graphs)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = eng.run_batches([24] * steps, task="transcribe", max_new_tokens=128, max_passes=1)
        torch.cuda.synchronize()
        res[beside].append(1000 * (time.perf_counter() - t0) / steps)
        toks[beside] = out[-1]
for k, v in res.items():
    print(json.dumps({"gemm_beside": k, "ms_per_step": [round(x, 2) for x in v], "min": round(min(v), 2)}))

"""Interleaved A/B of encoder-attention configurations in the bench workload (config 2: 24 windows, 128 tokens,
overlapped pipeline), one process: each config is (kernel alone, kernel beside, pad alone, pad beside).
    python scripts/exp/ab_attn_bench.py "10,10,0,4" "16,16,0,4" ..."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "turbo-whisper-workspace_amd")]
import torch  # noqa: E402

from twamd.config import PRESETS, GenerationSettings  # noqa: E402
from twamd.engine import WhisperEngine  # noqa: E402
from twamd.synth_audio import workload  # noqa: E402
from twamd.weights import build_weights  # noqa: E402

cfgs = [tuple(int(x) for x in c.split(",")) for c in sys.argv[1:]] or [(10, 10, 0, 4)]
steps, rounds = 8, 3
dims = PRESETS["large-v3-turbo"]
gen = GenerationSettings.default(dims)
eng = WhisperEngine(build_weights(dims, seed=1234), gen, max_batch=24, device="cuda:0")
eng.set_suppress_tokens(list(gen.suppress_tokens) + [gen.special.eot])
eng.wave[:24].copy_(torch.from_numpy(workload(24, 30.0, seed=1234)))
res = {c: [] for c in cfgs}
toks = {}
for r in range(rounds):
    for c in cfgs:
        eng.attn_kernel, eng.attn_pad = (c[0], c[1]), (c[2], c[3])
        eng.run_batches([24] * 2, task="transcribe", max_new_tokens=128, max_passes=1)  # warm (graphs)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = eng.run_batches([24] * steps, task="transcribe", max_new_tokens=128, max_passes=1)
        torch.cuda.synchronize()
        res[c].append(1000 * (time.perf_counter() - t0) / steps)
        toks[c] = out[-1]
for c, v in res.items():
    print(json.dumps({"config": c, "ms_per_step": [round(x, 2) for x in v], "min": round(min(v), 2),
                      "same_tokens_as_first": toks[c] == toks[cfgs[0]]}))

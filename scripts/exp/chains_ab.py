"""Experiment (not product code): does splitting a decode pass's rows into two chains replayed on two streams shorten
a decode pass that runs ALONE (no encoder beside it: config 3's per-rank share, the pipeline's last batch)?
Interleaved A/B of n_chains 1 vs 2 in one process, large-v3-turbo, EOS suppressed, 128 new tokens, one seek pass.

    python scripts/exp/chains_ab.py [--rows 15 24] [--rounds 3]
"""
import argparse
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


def set_chains(eng, k):
    eng.n_chains = k
    while len(eng._chain_streams) < k:
        s = torch.cuda.Stream(eng.device, priority=-1)
        eng._chain_streams.append(s)
        eng._own_streams.add(s.cuda_stream)
    eng._chain_streams = eng._chain_streams[:max(k, 1)]
    eng._chain_cache = {k_: v for k_, v in eng._chain_cache.items() if k_[0] != "chains"}
    eng._graphs = {k_: v for k_, v in eng._graphs.items() if k_[0] == "prompt"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, nargs="+", default=[15, 24])
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    d = PRESETS["large-v3-turbo"]
    gen = GenerationSettings.default(d)
    eng = WhisperEngine(build_weights(d, seed=1234), gen, max_batch=24)
    eng.set_suppress_tokens(list(gen.suppress_tokens) + [gen.special.eot])
    st = gen.special
    eng.wave[:24].copy_(torch.from_numpy(workload(24, 30.0, seed=1234)))
    for R in a.rows:
        eng.logmel(R)
        eng.row_map[:R] = torch.arange(R, dtype=torch.int32)
        eng.seek[:R] = 0
        eng.encode(R)
        torch.cuda.synchronize()
        res = {1: [], 2: []}
        toks = {}
        for r in range(a.rounds + 1):
            for k in (1, 2):
                set_chains(eng, k)
                eng.decode_pass(R, [st.transcribe], None, 128)  # captures this configuration's graphs
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                out = eng.decode_pass(R, [st.transcribe], None, 128)
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                if r:
                    res[k].append(dt * 1e3)
                toks[k] = out.tokens
        same = toks[1] == toks[2]
        print(f"R={R}: 1 chain {min(res[1]):.2f} ms (med {sorted(res[1])[len(res[1]) // 2]:.2f}), 2 chains "
              f"{min(res[2]):.2f} ms (med {sorted(res[2])[len(res[2]) // 2]:.2f}); tokens identical: {same}",
              flush=True)


if __name__ == "__main__":
    main()

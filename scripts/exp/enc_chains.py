"""Would two concurrent half-batch encoder chains fill each other's tails? The encoder of 24 windows on one engine
vs two 12-window engines encoding at once on their own streams (alone on the GPU; k_gemm_big or the 8-phase GEMM).

    python scripts/exp/enc_chains.py [--reps 5]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "turbo-whisper-workspace_amd")]
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    from twamd.config import PRESETS, GenerationSettings
    from twamd.engine import WhisperEngine
    from twamd.synth_audio import workload
    from twamd.weights import build_weights

    dims = PRESETS["large-v3-turbo"]
    gen = GenerationSettings.default(dims)
    w = build_weights(dims, seed=1234)
    audio = torch.from_numpy(workload(24, 30.0, seed=1234))
    full = WhisperEngine(w, gen, max_batch=24, device="cuda:0")
    halves = [WhisperEngine(w, gen, max_batch=12, device="cuda:0") for _ in range(2)]
    full.wave[:24].copy_(audio)
    for i, e in enumerate(halves):
        e.wave[:12].copy_(audio[12 * i:12 * (i + 1)])
    torch.cuda.synchronize()

    def one(alone_variant):
        for e in [full] + halves:
            e._gemm_alone = alone_variant
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        ev[0].record()
        full.logmel(24, sync=False)
        full.encode(24, row_map=False, seek=False, sync=False, alone=True)
        torch.cuda.current_stream().wait_stream(full.enc_stream)
        ev[1].record()
        torch.cuda.synchronize()
        ev[2].record()
        for e in halves:
            e.enc_stream.wait_stream(torch.cuda.current_stream())
        for e in halves:  # queued alternately so both chains are in flight
            e.logmel(12, sync=False)
        for e in halves:
            e.encode(12, row_map=False, seek=False, sync=False, alone=True)
        for e in halves:
            torch.cuda.current_stream().wait_stream(e.enc_stream)
        ev[3].record()
        torch.cuda.synchronize()
        return ev[0].elapsed_time(ev[1]), ev[2].elapsed_time(ev[3])

    for v in (1, 5):
        one(v)
        res = [one(v) for _ in range(a.reps)]
        f = sorted(r[0] for r in res)[len(res) // 2]
        h = sorted(r[1] for r in res)[len(res) // 2]
        print(f"gemm variant {v}: one 24-window chain {f:.2f} ms, two 12-window chains {h:.2f} ms", flush=True)


if __name__ == "__main__":
    main()

"""Stream timeline of the bench workload without a profiler (rocprofv3's kernel trace serialises the two streams):
every torch.cuda.Event the engine records (decode-step events of decode_pass, encoder-chunk events of the pump,
the per-slot encoder-done events) is made timing-enabled and logged with its recording site; afterwards the
per-batch picture is printed: decode span, encoder chunks finished inside it, encoder tail after it.

    python scripts/exp/timeline_events.py [--steps 3] [--batch 24]
"""
import argparse
import collections
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "turbo-whisper-workspace_amd"))
import torch  # noqa: E402

LOG = []
_Base = torch.cuda.Event


class TEvent(_Base):
    def __new__(cls, enable_timing=False, blocking=False, interprocess=False):
        return super().__new__(cls, enable_timing=True, blocking=blocking, interprocess=interprocess)

    def record(self, stream=None):
        super().record(stream)
        f = sys._getframe(1)
        LOG.append((f.f_code.co_name, time.perf_counter(), self))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--batch", type=int, default=24)
    ap.add_argument("--tokens", type=int, default=128)
    a = ap.parse_args()
    torch.cuda.Event = TEvent
    from twamd.config import PRESETS, GenerationSettings
    from twamd.engine import WhisperEngine
    from twamd.synth_audio import workload
    from twamd.weights import build_weights

    dims = PRESETS["large-v3-turbo"]
    gen = GenerationSettings.default(dims)
    B = a.batch
    eng = WhisperEngine(build_weights(dims, seed=1234), gen, max_batch=B, device="cuda:0")
    eng.set_suppress_tokens(list(gen.suppress_tokens) + [gen.special.eot])
    eng.wave[:B].copy_(torch.from_numpy(workload(B, 30.0, seed=1234)))
    eng.run_batches([B] * 2, task="transcribe", max_new_tokens=a.tokens, max_passes=1)
    torch.cuda.synchronize()
    LOG.clear()
    t0 = time.perf_counter()
    eng.run_batches([B] * a.steps, task="transcribe", max_new_tokens=a.tokens, max_passes=1)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ref = LOG[0][2]
    ev = [(site, h - t0, ref.elapsed_time(e)) for site, h, e in LOG]
    print(f"wall {wall * 1e3:.1f} ms for {a.steps} batches ({wall * 1e3 / a.steps:.1f} ms/batch); "
          f"{len(ev)} events; sites {dict(collections.Counter(s for s, _, _ in ev))}")
    # decode passes: runs of decode_pass events separated by > 3 ms
    dec = [(h, g) for s, h, g in ev if s == "decode_pass"]
    enc = [(h, g) for s, h, g in ev if s == "_one"]
    done = [(h, g) for s, h, g in ev if s == "_enc_end"]
    passes, cur = [], []
    for h, g in dec:
        if cur and g - cur[-1][1] > 3.0:
            passes.append(cur)
            cur = []
        cur.append((h, g))
    if cur:
        passes.append(cur)
    for i, p in enumerate(passes):
        g0, g1 = p[0][1], p[-1][1]
        inside = [g for h, g in enc if g0 <= g <= g1]
        after = [g for h, g in enc if g1 < g < (passes[i + 1][0][1] if i + 1 < len(passes) else 1e18)]
        steps = [p[j + 1][1] - p[j][1] for j in range(len(p) - 1)]
        steps.sort()
        med = steps[len(steps) // 2] if steps else 0
        print(f"pass {i}: gpu {g0:8.2f} -> {g1:8.2f} ms ({g1 - g0:6.2f} ms, {len(p)} step events, median step "
              f"{med * 1e3:.0f} us); encoder chunks done inside {len(inside)}, after {len(after)}"
              + (f" (last at {after[-1]:.2f}, tail {after[-1] - g1:.2f} ms)" if after else ""))
        host = [h for h, g in p]
        print(f"         host {host[0] * 1e3:8.2f} -> {host[-1] * 1e3:8.2f} ms")
    # encoder chunk completion spacing inside vs outside decode passes
    spans = [(p[0][1], p[-1][1]) for p in passes]

    def in_dec(g):
        return any(a0 <= g <= a1 for a0, a1 in spans)

    gaps_in, gaps_out = [], []
    for j in range(1, len(enc)):
        d = enc[j][1] - enc[j - 1][1]
        (gaps_in if in_dec(enc[j][1]) else gaps_out).append(d)
    for name, gs in (("inside decode", gaps_in), ("outside decode", gaps_out)):
        if gs:
            gs.sort()
            print(f"encoder chunk spacing {name}: n={len(gs)} median {gs[len(gs) // 2]:.3f} ms "
                  f"mean {sum(gs) / len(gs):.3f} ms")
    print("done events:", [round(g, 2) for h, g in done])


if __name__ == "__main__":
    main()

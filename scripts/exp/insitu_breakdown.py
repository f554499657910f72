"""Per-kernel cost of one captured decoder step (24 rows, large-v3-turbo) alone and beside a running encoder GEMM
stream, without a profiler (rocprofv3's kernel trace serialises the two streams): the step is captured as a hipGraph
with a timing event after every launch, so each event-to-event interval is that launch's cost in the replayed step
(execution + the boundary before it).

    python scripts/exp/insitu_breakdown.py [--variant 1] [--reps 20]
"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "turbo-whisper-workspace_amd")]
import torch  # noqa: E402

from twamd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", type=int, default=1)   # encoder GEMM kernel beside the decode
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--epi", type=int, default=1)       # encoder GEMM epilogue (1 = GELU fc1 shape, 2 = RESID fc2)
    ap.add_argument("--compute-only", action="store_true")  # storm of 8192 x 8192 x 4096 GEMMs (1024 tiles, operands resident in the Infinity Cache)
    a = ap.parse_args()
    from twamd.config import PRESETS, GenerationSettings
    from twamd.engine import WhisperEngine
    from twamd.synth_audio import workload
    from twamd.weights import build_weights

    dims = PRESETS["large-v3-turbo"]
    gen = GenerationSettings.default(dims)
    B = 24
    eng = WhisperEngine(build_weights(dims, seed=1234), gen, max_batch=B, device="cuda:0")
    eng.set_suppress_tokens(list(gen.suppress_tokens) + [gen.special.eot])
    eng.wave[:B].copy_(torch.from_numpy(workload(B, 30.0, seed=1234)))
    eng.run_batches([B] * 2, task="transcribe", max_new_tokens=8, max_passes=1)  # both slots encoded, state primed
    torch.cuda.synchronize()
    eng.use_slot(1)
    params = eng._select_params(0, 128, True)
    v = eng._chains(B)[0]
    st = v.stream

    # one fused decode step launched eagerly with a timing event after every C-ABI call (HIP graphs cannot hold
    # timing events); the steps are queued behind a gate (a sleep kernel on another stream) so the host is far
    # ahead and every event-to-event interval is GPU time: that launch's execution + the boundary before it
    marks = []
    orig = _lib.call
    rec = [False]

    def call(name, *args):
        r = orig(name, *args)
        if rec[0]:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record(st)
            marks[-1].append((name, ev))
        return r

    _lib.call = call
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        eng._embed_head(v)
    torch.cuda.synchronize()
    # every step restarts from the same decoder position/state (a step advances pos, ngen and the KV cache append
    # point: without the reset they would run past max_target_positions)
    saved = {k: getattr(v, k).clone() for k in ("state", "pos", "ids", "xd", "hp")}
    aux = torch.cuda.Stream()

    def replay(n):
        marks.clear()
        gate = torch.cuda.Event()
        with torch.cuda.stream(aux):
            torch.cuda._sleep(200_000_000)  # ~0.1 s at ~2 GHz: the host queues all n steps meanwhile
            gate.record(aux)
        st.wait_event(gate)
        starts = []
        with torch.cuda.stream(st):
            for _ in range(n):
                for k, t in saved.items():
                    getattr(v, k).copy_(t)
                e = torch.cuda.Event(enable_timing=True)
                e.record(st)
                starts.append(e)
                marks.append([])
                rec[0] = True
                eng._gen_step(B, params, v=v, r_enc=B, fused=True)
                rec[0] = False
        st.synchronize()
        per = collections.defaultdict(list)
        tot = []
        for e, ms in zip(starts, marks):
            prev = e
            for nm, ev in ms:
                per[nm].append(prev.elapsed_time(ev) * 1e3)
                prev = ev
            tot.append(e.elapsed_time(ms[-1][1]) * 1e3)
        return per, tot

    replay(3)
    alone, tot_a = replay(a.reps)
    # encoder GEMM storm on a default-priority stream (the engine's enc_stream), then replay the step inside it
    M, D, F = B * 1500, 1280, 5120
    N, K = (F, D) if a.epi == 1 else (D, F)
    if a.compute_only:  # operands stay in the Infinity Cache / L2, 8 MB of output per launch: MFMA work, little HBM
        M, N, K = 8192, 8192, 4096
    A = (torch.randn(M, K, device="cuda") * 0.5).to(torch.bfloat16)
    W = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
    out = torch.empty(M, N, dtype=torch.bfloat16 if a.epi == 1 else torch.float32, device="cuda")
    bias = torch.zeros(N, device="cuda")
    es = eng.enc_stream
    orig("tw_gemm_set_variant", a.variant)
    for _ in range(1000 if a.compute_only else 600):  # (the storm must outlast the 0.1 s gate + the steps)
        orig("tw_gemm_bf16", A.data_ptr(), W.data_ptr(), M, N, K, K, K, a.epi, out.data_ptr(), N,
                  bias.data_ptr(), None, 0, None, es.cuda_stream)
    done = torch.cuda.Event()
    done.record(es)
    beside, tot_b = replay(a.reps)
    beside_done = done.query()  # the storm must still be running when the last step ends
    torch.cuda.synchronize()
    _lib.call = orig

    def med(x):
        x = sorted(x)
        return x[len(x) // 2] if x else float("nan")

    print(f"step: alone median {med(tot_a):.1f} us, beside GEMM variant {a.variant} median {med(tot_b):.1f} us "
          f"({len(tot_b)} steps; GEMM stream still busy at the end: {not beside_done})")
    counts = collections.Counter(nm for nm, _ in marks[0])
    print(f"{'kernel (C-ABI call)':32s} {'n/step':>6s} {'alone us':>9s} {'beside us':>10s} {'delta/step':>10s}")
    rows = []
    for nm, c in counts.items():
        al, bs = med(alone[nm]), med(beside[nm])
        rows.append((c * (bs - al), nm, c, al, bs))
    for d, nm, c, al, bs in sorted(rows, reverse=True):
        print(f"{nm:32s} {c:6d} {al:9.2f} {bs:10.2f} {d:10.1f}")


if __name__ == "__main__":
    main()

"""Measurement (not a bench line): what each kernel family of the captured greedy decoder step costs IN the chain.

For R rows at large-v3-turbo dims, one decoder step + fused selection is captured as a hipGraph and replayed; then
the same step is captured with one kernel family left out (its launches not issued: the outputs are stale, the
timing is what matters), and the difference is that family's marginal cost per step — what fusing it away could
save at most. A chain of trivial kernels of the same length gives the boundary floor. Prints one JSON line per case.

    python scripts/decode_chain_costs.py [--rows 24] [--reps 300]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "turbo-whisper-workspace_amd")]
import torch  # noqa: E402

from twamd import _lib  # noqa: E402
from twamd.config import PRESETS, GenerationSettings  # noqa: E402
from twamd.engine import WhisperEngine  # noqa: E402
from twamd.synth_audio import workload  # noqa: E402
from twamd.weights import build_weights  # noqa: E402

SKIP = set()
_real_call = _lib.call


def _call(name, *args):
    if name in SKIP:
        return
    _real_call(name, *args)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, nargs="+", default=[24])
    ap.add_argument("--reps", type=int, default=300)
    ap.add_argument("--pos", type=int, default=64)
    ap.add_argument("--variants", type=int, nargs="+", default=[0], help="tw_gemv_set_variant values to compare")
    ap.add_argument("--families", type=int, default=1, help="0: the full step only")
    ap.add_argument("--passlike", type=int, default=0)
    ap.add_argument("--wide-kw", type=int, nargs="+", default=[1], help="proj_out K-slices (tw_gemv_set_wide_slices)")
    a = ap.parse_args()
    dims = PRESETS["large-v3-turbo"]
    gen = GenerationSettings.default(dims)
    B = max(a.rows)
    eng = WhisperEngine(build_weights(dims, seed=1234), gen, max_batch=B, device="cuda")
    eng.set_suppress_tokens(list(gen.suppress_tokens) + [gen.special.eot])
    eng.wave[:B].copy_(torch.from_numpy(workload(B, 30.0, seed=1234)))
    eng.logmel(B)
    _lib.call = _call
    D, F = dims.d_model, dims.ffn
    gemv_kind = {}

    real_gemv = eng._gemv

    def gemv(A, a_packed, Wp, M, N, K, epi, out, v, bias=None, splits=1, ldo=None):
        kind = {(3 * D, D): "qkv", (D, F): "fc2", (F, D): "fc1"}.get((N, K))
        if kind is None:
            kind = "proj_out" if N == dims.vocab else ("o_proj" if epi == _lib.TW_EPI_PARTIAL_F32 else "q_x")
        gemv_kind[kind] = gemv_kind.get(kind, 0) + 1
        if kind in SKIP:
            return
        real_gemv(A, a_packed, Wp, M, N, K, epi, out, v, bias=bias, splits=splits, ldo=ldo)

    eng._gemv = gemv
    for R in a.rows:
        eng.row_map[:R] = torch.arange(R, dtype=torch.int32)
        eng.seek[:R] = 0
        eng.encode(R)
        torch.cuda.synchronize()
        params = eng._select_params(0, 448 - 8)

        def step():
            eng.pos[:R] = a.pos
            eng.state[:R].zero_()
            eng._gen_step(R, params, fused=True)

        def timed(fn, label, n_launch=None):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.stream(eng.stream):
                fn()  # warm (eager)
                torch.cuda.synchronize()
                with torch.cuda.graph(g, stream=eng.stream):
                    fn()
                for _ in range(20):
                    g.replay()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(eng.stream)
                for _ in range(a.reps):
                    g.replay()
                e1.record(eng.stream)
                torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / a.reps
            return us

        ref_logits = None
        for var, wkw in [(v_, w_) for w_ in a.wide_kw for v_ in a.variants]:
            _real_call("tw_gemv_set_variant", var)
            _real_call("tw_gemv_set_wide_slices", wkw)
            with torch.cuda.stream(eng.stream):
                eng.ids[:R] = 50300
                eng.pos[:R] = a.pos
                eng._embed_head(eng._view(0, R))
                eng.decoder_step(R, pre_embedded=True)
            torch.cuda.synchronize()
            lg = eng.logits[:R].clone()
            if ref_logits is None:
                ref_logits = lg
            diff = float((lg - ref_logits).abs().max())
            base = timed(step, "full")
            print(json.dumps({"rows": R, "gemv_variant": var, "wide_kw": wkw, "case": "full step", "us": round(base, 1),
                              "logits_maxdiff_vs_first": diff}), flush=True)
        if a.passlike:
            # the step graph replayed as a pass replays it: positions advancing from 3, state carried (pass-like),
            # against the same with the position reset every step (fixed) or the state zeroed every step
            chain = eng._chains(R)[0]
            for label, reset_pos, zero_state, view in (("advancing pos, state carried", False, False, None),
                                                        ("advancing pos, state zeroed", False, True, None),
                                                        ("fixed pos, state carried", True, False, None),
                                                        ("chain view + stream", False, False, chain)):
                def stp(reset_pos=reset_pos, zero_state=zero_state, view=view):
                    if reset_pos:
                        eng.pos[:R] = a.pos
                    if zero_state:
                        eng.state[:R].zero_()
                    eng._gen_step(R, params, v=view, r_enc=R, fused=True)
                g = torch.cuda.CUDAGraph()
                st = eng.stream if view is None else view.stream
                st.wait_stream(eng.stream)
                with torch.cuda.stream(st):
                    eng.pos[:R] = 3
                    eng.state[:R].zero_()
                    stp()
                    torch.cuda.synchronize()
                    with torch.cuda.graph(g, stream=st):
                        stp()
                    eng.pos[:R] = 3
                    eng.state[:R].zero_()
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(st)
                    th = time.perf_counter()
                    for _ in range(127):
                        g.replay()
                    th = time.perf_counter() - th
                    e1.record(st)
                    torch.cuda.synchronize()
                print(json.dumps({"rows": R, "case": label, "us": round(e0.elapsed_time(e1) * 1e3 / 127, 1),
                                  "host_us_per_replay": round(th * 1e6 / 127, 1), "final_pos": int(eng.pos[0])}),
                      flush=True)
        if a.passlike:
            # the graph decode_pass itself captured, replayed by this loop; then decode_pass's own loop (events)
            tail = eng.prompt_tail("transcribe", True)
            eng._graphs.clear()
            eng.decode_pass(R, tail, None, 128, check_every=128)
            torch.cuda.synchronize()
            keys = [k for k in eng._graphs if k[0] == R]
            st = eng._chains(R)[0].stream
            for k in keys:
                g = eng._graphs[k]
                with torch.cuda.stream(st):
                    eng.pos[:R] = 3
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(st)
                    for _ in range(127):
                        g.replay()
                    e1.record(st)
                    torch.cuda.synchronize()
                print(json.dumps({"rows": R, "case": "decode_pass graph " + str(k[:6]),
                                  "us": round(e0.elapsed_time(e1) * 1e3 / 127, 1)}), flush=True)
            # decode_pass's loop body, replayed here: per-step stream context around the replay
            g = eng._graphs[keys[0]]
            with torch.cuda.stream(st):
                eng.pos[:R] = 3
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            th = time.perf_counter()
            for _ in range(127):
                with torch.cuda.stream(st):
                    g.replay()
            th = time.perf_counter() - th
            e1.record(st)
            torch.cuda.synchronize()
            print(json.dumps({"rows": R, "case": "per-step stream context", "us": round(e0.elapsed_time(e1) * 1e3 / 127, 1),
                              "host_us": round(th * 1e6 / 127, 1)}), flush=True)
            # the same from inside the engine's stream wrapper (decode_pass runs under on_engine_streams)
            with torch.cuda.stream(eng.stream):
                eng.pos[:R] = 3
                torch.cuda.synchronize()
                e0.record(st)
                th = time.perf_counter()
                for _ in range(127):
                    with torch.cuda.stream(st):
                        g.replay()
                th = time.perf_counter() - th
                e1.record(st)
                torch.cuda.synchronize()
            print(json.dumps({"rows": R, "case": "inside eng.stream", "us": round(e0.elapsed_time(e1) * 1e3 / 127, 1),
                              "host_us": round(th * 1e6 / 127, 1)}), flush=True)
            # decode_pass's structure rebuilt step by step: (A) prompt graph on eng.stream, head on the chain stream,
            # 127 replays; (B) the same without the prompt graph
            pk = [k for k in eng._graphs if k[0] == "prompt"]
            c = eng._chains(R)[0]
            def plain(label):
                with torch.cuda.stream(eng.stream):
                    eng.pos[:R] = 3
                    torch.cuda.synchronize()
                    e0.record(st)
                    for _ in range(127):
                        with torch.cuda.stream(st):
                            g.replay()
                    e1.record(st)
                    torch.cuda.synchronize()
                print(json.dumps({"rows": R, "case": label, "us": round(e0.elapsed_time(e1) * 1e3 / 127, 1)}),
                      flush=True)

            plain("plain again")

            def variant(label, wait, head, sync, e1_on_eng):
                torch.cuda.synchronize()
                with torch.cuda.stream(eng.stream):
                    eng.pos[:R] = 3
                    if wait:
                        c.stream.wait_stream(eng.stream)
                    if head:
                        with torch.cuda.stream(c.stream):
                            eng._embed_head(c)
                    if sync:
                        torch.cuda.synchronize()
                    e0.record(c.stream)
                    for _ in range(127):
                        with torch.cuda.stream(c.stream):
                            g.replay()
                    if e1_on_eng:
                        eng.stream.wait_stream(c.stream)
                        e1.record(eng.stream)
                    else:
                        e1.record(c.stream)
                torch.cuda.synchronize()
                print(json.dumps({"rows": R, "case": label, "us": round(e0.elapsed_time(e1) * 1e3 / 127, 1)}),
                      flush=True)

            variant("B  wait+head, no sync, e1 on eng", True, True, False, True)
            variant("B1 wait, no head, no sync, e1 on eng", True, False, False, True)
            variant("B2 wait+head, sync", True, True, True, True)
            variant("B3 head, no wait, no sync", False, True, False, True)
            variant("B4 wait, sync, no head", True, False, True, True)
            variant("B5 wait+head, no sync, e1 on chain", True, True, False, False)
            variant("B6 nothing, no sync, e1 on chain", False, False, False, False)
            plain("plain after")
            with torch.cuda.stream(eng.stream):
                eng.state[:R].zero_()
            plain("plain, state zeroed")
            plain("plain, state carried on")
            eng.pass_events = []
            for _ in range(3):
                eng.decode_pass(R, tail, None, 128, check_every=128)
            torch.cuda.synchronize()
            print(json.dumps({"rows": R, "case": "decode_pass loop", "us": [
                (round(e0.elapsed_time(e1) * 1e3 / n, 1), round(th * 1e6 / n, 1)) for e0, e1, n, th in eng.pass_events]}), flush=True)
            eng.pass_events = None
            import numpy as np
            rh = np.array(eng.replay_host[-127:]) * 1e6
            print(json.dumps({"replay_host_us": {"mean": round(float(rh.mean()), 1), "p50": round(float(np.median(rh)), 1),
                              "max": round(float(rh.max()), 1), "first8": [round(float(x), 1) for x in rh[:8]]}}))
        if not a.families:
            continue
        # a chain of trivial kernels as long as the step (47 launches + the two state writes)
        tiny = torch.zeros(64, device="cuda")

        def trivial(n=49):
            for _ in range(n):
                tiny.add_(1.0)

        t_triv = timed(trivial, "trivial")
        print(json.dumps({"rows": R, "case": "49 trivial kernels", "us": round(t_triv, 1),
                          "per_launch_us": round(t_triv / 49, 2)}), flush=True)
        fams = [
            ("resid_ln", {"tw_resid_layernorm_packed"}),
            ("self_attn", {"tw_attn_decode_self"}),
            ("cross_attn", {"tw_attn_decode_cross"}),
            ("select_embed", {"tw_logits_select_embed"}),
            ("qkv", {"qkv"}), ("o_proj", {"o_proj"}), ("q_x", {"q_x"}), ("fc1", {"fc1"}), ("fc2", {"fc2"}),
            ("proj_out", {"proj_out"}),
        ]
        for label, names in fams:
            SKIP.clear()
            SKIP.update(names)
            t = timed(step, label)
            SKIP.clear()
            print(json.dumps({"rows": R, "case": f"without {label}", "us": round(t, 1),
                              "saved_us": round(base - t, 1)}), flush=True)


if __name__ == "__main__":
    main()

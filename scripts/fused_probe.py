"""Measurement (not a bench line): where one tw_dec_fused launch (the decoder's layers for one token as one persistent
launch, csrc/decfused.hip) spends its time, from the kernel's own per-workgroup timestamps (tw_dec_fused_set_probe):
per layer and phase the first / median / last workgroup start (after its wait) and end, in us from the first
workgroup's start, and the hand-off gap (first start of a phase - last end of the phase it waits for). Rows of
large-v3-turbo dims, random caches and cross K/V, positions at --pos.

    python scripts/fused_probe.py [--rows 15] [--pos 64] [--steps 5] [--acquire 0]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "turbo-whisper-workspace_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from twamd import _lib  # noqa: E402
from twamd.config import PRESETS, GenerationSettings  # noqa: E402
from twamd.engine import WhisperEngine  # noqa: E402
from twamd.weights import build_weights  # noqa: E402

KINDS = ["ln1", "qkv", "self", "o", "ln2", "qx", "cross", "ox", "ln3", "fc1", "fc2", "fin"]
NK = len(KINDS)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=15)
    ap.add_argument("--pos", type=int, default=64)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--acquire", type=int, default=0)
    a = ap.parse_args()
    dims = PRESETS["large-v3-turbo"]
    R = a.rows
    eng = WhisperEngine(build_weights(dims, seed=1234), GenerationSettings.default(dims), max_batch=R, device="cuda")
    g = torch.Generator(device=eng.device).manual_seed(7)
    for t in (eng.kcache, eng.vcache, eng.cross_kv):
        t.copy_(torch.randn(t.shape, generator=g, device=eng.device) * 0.5)
    eng.pos[:R] = a.pos
    eng.ids[:R] = torch.arange(R, dtype=torch.int32, device=eng.device) + 1000
    eng.dec_fused_alone = True
    eng._dec_context()
    _lib.call("tw_dec_fused_set_acquire", a.acquire)
    eng.decoder_step(R)  # warm-up (grid query)
    torch.cuda.synchronize()
    G = int(_lib.load().tw_dec_fused_grid())
    L = dims.decoder_layers
    buf = torch.zeros((L + 1) * NK * G * 2, dtype=torch.int64, device=eng.device)
    _lib.call("tw_dec_fused_set_probe", buf.data_ptr())
    per = []
    try:
        for _ in range(a.steps):
            buf.zero_()
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record(eng.stream)
            eng.decoder_step(R)
            ev1.record(eng.stream)
            torch.cuda.synchronize()
            t = buf.view(L + 1, NK, G, 2).cpu().numpy().astype(np.float64)
            per.append((t, ev0.elapsed_time(ev1) * 1e3))
    finally:
        _lib.call("tw_dec_fused_set_probe", None)
    # the step's launches timed apart with HIP events on the engine stream: embedding, tw_dec_fused (memset node +
    # kernel), proj_out
    v = eng._view(0, R)
    d = eng.d
    parts = {"embed": [], "fused": [], "proj_out": []}
    for _ in range(a.steps):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        with torch.cuda.stream(eng.stream):
            ev[0].record(eng.stream)
            _lib.call("tw_embed_decoder", eng.w.emb.data_ptr(), eng.w.pos_dec.data_ptr(), v.ids.data_ptr(),
                      v.pos.data_ptr(), R, d.d_model, v.xd.data_ptr(), eng.stream.cuda_stream)
            ev[1].record(eng.stream)
            eng._fused_layers(R, R, v)
            ev[2].record(eng.stream)
            eng._gemv(v.hp, True, eng.emb_p, R, d.vocab, d.d_model, _lib.TW_EPI_F32, v.logits, v)
            ev[3].record(eng.stream)
        torch.cuda.synchronize()
        for k, (i, j) in zip(parts, ((0, 1), (1, 2), (2, 3))):
            parts[k].append(ev[i].elapsed_time(ev[j]) * 1e3)
    print(json.dumps({"launch_us_median": {k: round(float(np.median(x)), 1) for k, x in parts.items()}}), flush=True)
    eng.check_fused()
    # the median step by kernel span
    spans = []
    for t, _ in per:
        starts = t[L, 0, :, 0]
        ends = t[:L, :, :, 1]
        spans.append((ends[ends > 0].max() - starts.min()) / 100.0)
    k = int(np.argsort(spans)[len(spans) // 2])
    t, step_us = per[k]
    t0 = t[L, 0, :, 0].min()
    us = lambda v: round((v - t0) / 100.0, 2)  # noqa: E731
    print(json.dumps({"rows": R, "pos": a.pos, "grid": G, "acquire": a.acquire, "kernel_span_us": round(spans[k], 1),
                      "step_events_us": round(step_us, 1), "wg_start_spread_us": us(t[L, 0, :, 0].max())}), flush=True)
    prev_end = None
    for li in range(L + 1):
        for ki, name in enumerate(KINDS):
            if li == L and name != "fin":
                continue
            if li < L and name == "fin":
                continue
            s, e = t[li, ki, :, 0], t[li, ki, :, 1]
            m = (s > 0) & (e > 0)
            if not m.any():
                continue
            s, e = s[m], e[m]
            row = {"layer": li, "phase": name, "wgs": int(m.sum()), "start_first": us(s.min()),
                   "start_med": us(np.median(s)), "start_last": us(s.max()), "end_first": us(e.min()),
                   "end_med": us(np.median(e)), "end_last": us(e.max()),
                   "work_med_us": round(float(np.median(e - s)) / 100.0, 2)}
            if prev_end is not None:
                row["gap_us"] = round((s.min() - prev_end) / 100.0, 2)
            prev_end = e.max()
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()

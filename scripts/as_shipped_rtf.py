"""Measurement (not a bench line): the drop-in as from_pretrained builds it by default (24-window engine batches,
beam-5 rows) with the reference's exact call (chunk_length_s=60, stride_length_s=5, batch_size=32,
generate_kwargs={"task": "transcribe"}, return_timestamps=True) on N minutes of synthetic speech, large-v3-turbo,
seeded synthetic weights, one GPU: wall time per call after one warm-up call, and the same with num_beams=1.
--fused 1: the transcriber built with fused_decode=True (the persistent decoder launch for greedy passes of <= 4 rows)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "turbo-whisper-workspace_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from twamd.pipeline import TurboTranscriber  # noqa: E402
from twamd.synth_audio import speech_like  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--minutes", type=float, default=10.0)
ap.add_argument("--model", default="large-v3-turbo", help="large-v3: the reference's own default model "
                "(vocalis/core/audio_pipeline.py:171), the turbo encoder with a 32-layer decoder")
ap.add_argument("--fused", type=int, default=0)
ap.add_argument("--modes", default="as_shipped_beam5,greedy", help="which calls to time (comma-separated)")
a = ap.parse_args()
tr = TurboTranscriber.from_pretrained(a.model, seed=1234, fused_decode=bool(a.fused))
audio = np.concatenate([speech_like(60.0, 500 + i) for i in range(int(a.minutes))]).astype(np.float32)
kw = dict(chunk_length_s=60, stride_length_s=5, batch_size=32, return_timestamps=True)
out = {}
for name, gk in (("as_shipped_beam5", {"task": "transcribe"}), ("greedy", {"task": "transcribe", "num_beams": 1})):
    if name not in a.modes.split(","):
        continue
    tr(audio, generate_kwargs=dict(gk), **kw)  # warm-up (graph captures, buffers)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = tr(audio, generate_kwargs=dict(gk), **kw)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    out[name] = {"wall_s": round(dt, 3), "rtf": round(len(audio) / 16000 / dt, 1), "chunks": len(r["chunks"])}
    print(name, out[name], flush=True)
print(json.dumps({"model": a.model, "fused_decode": bool(a.fused), "audio_s": len(audio) / 16000,
                  "windows_60_5": len(tr.last_window_passes), **out}))

"""Measurement (not a bench line): native Ogg Vorbis decode speed on the host cores, by thread count, on a random-
syntax stream from the oracle's writer (44.1 kHz stereo, 256 / 2048 blocks, 200-400-byte packets: libvorbis-q5-like
packet sizes). Prints one JSON line per thread count: audio seconds decoded per wall second."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "turbo-whisper-workspace_amd")]
import numpy as np  # noqa: E402

from oracle import vorbis_oracle as vo  # noqa: E402
from twamd import audio  # noqa: E402

data = vo.write_stream(np.random.default_rng(1), channels=2, bs_exp=(8, 11), n_packets=6000, rate=44100,
                       packet_bytes=(200, 400))
secs = audio.vorbis_probe(data).total_samples / 44100
for th in (1, 4, 8, 16):
    audio.decode_vorbis(data, threads=th)
    t = time.perf_counter()
    for _ in range(3):
        audio.decode_vorbis(data, threads=th)
    dt = (time.perf_counter() - t) / 3
    print(json.dumps({"threads": th, "audio_s": round(secs, 2), "wall_ms": round(dt * 1e3, 1),
                      "x_realtime": round(secs / dt, 1)}), flush=True)

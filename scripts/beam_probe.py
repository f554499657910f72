"""Measurement aid (not a bench line; needs the -DTW_BEAM_PROBE library, `make -C turbo-whisper-workspace_amd/csrc
beamprobe`, copied over twamd/libtwhip.so on the box): the as-shipped beam-5 call (scripts/as_shipped_rtf.py), then
the per-phase timestamps of block 0 of the last k_beam_partial / k_beam_step launches (100 MHz s_memrealtime)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "turbo-whisper-workspace_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from twamd import _lib  # noqa: E402
from twamd.pipeline import TurboTranscriber  # noqa: E402
from twamd.synth_audio import speech_like  # noqa: E402

minutes = float(sys.argv[1]) if len(sys.argv) > 1 else 2.0
tr = TurboTranscriber.from_pretrained("large-v3-turbo", seed=1234)
audio = np.concatenate([speech_like(60.0, 500 + i) for i in range(int(minutes))]).astype(np.float32)
kw = dict(chunk_length_s=60, stride_length_s=5, batch_size=32, return_timestamps=True)
lib = _lib.load()
buf = (ctypes.c_ulonglong * 32)()
for rep in range(3):
    tr(audio, generate_kwargs={"task": "transcribe"}, **kw)
    torch.cuda.synchronize()
    assert lib.tw_beam_probe_read(buf) == 0
    ts = np.array(buf[:], np.int64).reshape(2, 16)
    for k, name, n in ((0, "k_beam_partial", 5), (1, "k_beam_step", 7)):
        t = ts[k, :n]
        print(name, "phase us:", [round((t[i + 1] - t[i]) / 100.0, 2) for i in range(n - 1)],
              "total", round((t[n - 1] - t[0]) / 100.0, 2), flush=True)
    t = ts[1]  # inside k_beam_step's step 1 (thread 0): loads + lse, text top-K, picks, staging
    print("  step1 detail us:", [round((b - a) / 100.0, 2) for a, b in ((t[1], t[8]), (t[8], t[9]), (t[9], t[11]),
                                                                      (t[11], t[2]))], flush=True)

"""Profiling driver (not product code): one warm and one timed as-shipped beam-5 call on 10 minutes of audio
(large-v3-turbo), reporting decode steps per window pass."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "turbo-whisper-workspace_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from twamd.pipeline import TurboTranscriber  # noqa: E402
from twamd.synth_audio import speech_like  # noqa: E402

tr = TurboTranscriber.from_pretrained("large-v3-turbo", seed=1234)
audio = np.concatenate([speech_like(60.0, 500 + i) for i in range(10)]).astype(np.float32)
kw = dict(chunk_length_s=60, stride_length_s=5, batch_size=32, return_timestamps=True)
for rep in range(2):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr(audio, generate_kwargs={"task": "transcribe"}, **kw)
    torch.cuda.synchronize()
    print(rep, round(time.perf_counter() - t0, 3), "s; passes per window:",
          [len(p) for p in tr.last_window_passes], "tokens per pass:",
          [[len(x) for x in p] for p in tr.last_window_passes][:3], flush=True)

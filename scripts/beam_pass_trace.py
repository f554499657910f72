"""Measurement aid (not a bench line): which engine passes the as-shipped call (scripts/as_shipped_rtf.py's beam-5
call) runs — windows, beams, max_new and the steps each pass took — to see where its decode steps go."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "turbo-whisper-workspace_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from twamd import engine as E  # noqa: E402
from twamd.pipeline import TurboTranscriber  # noqa: E402
from twamd.synth_audio import speech_like  # noqa: E402

minutes = float(sys.argv[1]) if len(sys.argv) > 1 else 10.0
model = sys.argv[2] if len(sys.argv) > 2 else "large-v3-turbo"
tr = TurboTranscriber.from_pretrained(model, seed=1234)
eng = tr.engine if hasattr(tr, "engine") else tr.eng
log = []
for name in ("beam_pass", "decode_pass", "sample_pass", "encode"):
    if not hasattr(E.WhisperEngine, name):
        continue
    orig = getattr(E.WhisperEngine, name)

    def wrap(self, *a, _orig=orig, _name=name, **k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = _orig(self, *a, **k)
        torch.cuda.synchronize()
        info = {"call": _name, "args": [x for x in a if isinstance(x, (int, float))][:4],
                "kw": {kk: v for kk, v in k.items() if isinstance(v, (int, float, bool))}, "ms": round(1e3 * (time.perf_counter() - t0), 2)}
        if _name == "beam_pass":
            info["win_t"] = self._beam["win"][:, 2].tolist()[:a[0]] if isinstance(a[0], int) else None
        log.append(info)
        return r
    setattr(E.WhisperEngine, name, wrap)
audio = np.concatenate([speech_like(60.0, 500 + i) for i in range(int(minutes))]).astype(np.float32)
kw = dict(chunk_length_s=60, stride_length_s=5, batch_size=32, return_timestamps=True)
tr(audio, generate_kwargs={"task": "transcribe"}, **kw)
log.clear()
t0 = time.perf_counter()
tr(audio, generate_kwargs={"task": "transcribe"}, **kw)
print("call ms", round(1e3 * (time.perf_counter() - t0), 1))
for x in log:
    print(x)
print("max_rows", eng.max_rows, "max_batch", eng.max_batch, "max_beams", eng.max_beams)
print("generation", {k: getattr(tr, k) for k in dir(tr) if "gen" in k.lower() and not k.startswith("__")}.keys())

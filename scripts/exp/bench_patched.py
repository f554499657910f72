"""Measurement helper (not a bench line): run bench.py with WhisperEngine attributes overridden after construction,
for A/B of engine switches that have no environment variable. TW_PATCH="fused_select=0,prompt_graph=1".

    python scripts/exp/bench_patched.py --steps 20 --warmup 5 --no-cpu-baseline
"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "turbo-whisper-workspace_amd")]

from twamd import engine  # noqa: E402

_init = engine.WhisperEngine.__init__


def _patched(self, *a, **k):
    _init(self, *a, **k)
    for kv in filter(None, os.environ.get("TW_PATCH", "").split(",")):
        key, val = kv.split("=")
        cur = getattr(self, key)
        setattr(self, key, type(cur)(int(val)) if isinstance(cur, (bool, int)) else val)


engine.WhisperEngine.__init__ = _patched
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[1:]
runpy.run_path(os.path.join(ROOT, "bench.py"), run_name="__main__")

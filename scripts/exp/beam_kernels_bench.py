"""Microbenchmark (not product code): tw_beam_step (k_beam_partial + k_beam_step) at the as-shipped beam-5 shape
(12 windows x 5 beams, vocab 51866) on random logits; optional library path argument (probe builds)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "turbo-whisper-workspace_amd")]
import torch  # noqa: E402

from twamd import _lib  # noqa: E402
from twamd.config import PRESETS, GenerationSettings  # noqa: E402

if len(sys.argv) > 1:
    _lib.load(sys.argv[1])
d = PRESETS["large-v3-turbo"]
gen = GenerationSettings.default(d)
st = gen.special
W, nb, V, T = 12, 5, d.vocab, 448
R = W * nb
dev = "cuda"
logits = torch.randn(R, V, device=dev) * 3
state = torch.zeros(R, _lib.TW_STATE_STRIDE, dtype=torch.int32, device=dev)
state[:, _lib.TW_ST_NGEN] = 5
tokens = torch.zeros(R, T, dtype=torch.int32, device=dev)
ids = torch.zeros(R, dtype=torch.int32, device=dev)
pos = torch.full((R,), 100, dtype=torch.int32, device=dev)
f32 = lambda n, v: torch.full((n,), v, dtype=torch.float32, device=dev)  # noqa: E731
run_score, fin_score = f32(R, 0.0), f32(R, -1e9)
fin_flag = torch.zeros(R, dtype=torch.int32, device=dev)
fin_len = torch.zeros(R, dtype=torch.int32, device=dev)
fin_tokens = torch.zeros(R, T, dtype=torch.int32, device=dev)
win = torch.tensor([[1, 0, 50, 0]] * W, dtype=torch.int32, device=dev)
src_rows = torch.zeros(R, dtype=torch.int32, device=dev)
ws = torch.empty(int(_lib.load().tw_beam_workspace_bytes(R)), dtype=torch.uint8, device=dev)
sup = torch.zeros((V + 31) // 32, dtype=torch.int32, device=dev)
bs_ = list(gen.begin_suppress_tokens)[:8]
sel = _lib.TwSelectParams(V, st.eot, st.eot, st.timestamp_begin, st.notimestamps, 50, 1, 440, 0, 0, 0,
                          len(bs_), (ctypes.c_int32 * 8)(*(bs_ + [0] * (8 - len(bs_)))))
bp = _lib.TwBeamParams(nb, 440, 1.0, T)
bst = _lib.TwBeamState(run_score.data_ptr(), fin_score.data_ptr(), fin_flag.data_ptr(), fin_len.data_ptr(),
                       fin_tokens.data_ptr(), win.data_ptr(), src_rows.data_ptr(), None)
s = torch.cuda.current_stream().cuda_stream


def call():
    win[:, 2] = 50
    pos.fill_(100)
    _lib.call("tw_beam_step", logits.data_ptr(), W, V, sup.data_ptr(), ctypes.byref(sel), ctypes.byref(bp),
              ctypes.byref(bst), state.data_ptr(), tokens.data_ptr(), ids.data_ptr(), pos.data_ptr(), ws.data_ptr(), s)


for _ in range(20):
    call()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(200):
    call()
e1.record()
torch.cuda.synchronize()
print(f"{sys.argv[1] if len(sys.argv) > 1 else 'product'}: {e0.elapsed_time(e1) / 200 * 1000:.1f} us per tw_beam_step "
      "(incl. two tiny torch fills)", flush=True)

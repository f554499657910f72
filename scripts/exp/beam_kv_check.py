"""Diagnostic (not product code): run the engine's beam search step by step on sweep case nochunk_beam5 and, after every
decoder step, compare each running beam row's logits with a fresh teacher-forced computation of that row's token
history on a second engine: the first step where they differ locates a history / K-V bookkeeping fault."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "turbo-whisper-workspace_amd"), os.path.join(ROOT, "tests", "golden")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from make_golden import sweep_audio  # noqa: E402
from twamd import _lib  # noqa: E402
from twamd.pipeline import TurboTranscriber  # noqa: E402

audio = sweep_audio([("speech", 25.0, 36)])
A = TurboTranscriber.from_pretrained("test-mini", seed=1234, max_batch=8, max_beams=5).engine
B = TurboTranscriber.from_pretrained("test-mini", seed=1234, max_batch=8, max_beams=1).engine
st = A.gen.special
host = np.zeros((1, 480000), np.float32)
host[0, : len(audio)] = audio[:480000]
for e in (A, B):
    e.wave[:1].copy_(torch.from_numpy(host))
    e.logmel(1)
    e.row_map[0] = 0
    e.seek[0] = 0
    e.encode(1)

nb, W, R = 5, 1, 5
max_new = 24
res = A.generate(1, task="transcribe", max_new_tokens=max_new, num_beams=5, max_passes=1)
print("engine generate:", A.last_passes[0][0])
# manual replica of beam_pass with checks
A.logmel(1)
A.row_map[0] = 0
A.seek[0] = 0
A.encode(1)
lang = A.last_langs[0]
prompt = [st.sot, lang, st.transcribe]


def tf_logits(hist):
    full = prompt + hist
    for p_, tok in enumerate(full):
        B.ids[0] = tok
        B.pos[0] = p_
        B.decoder_step(1)
    return B.logits[0].float().cpu().numpy()


bb = A._beam_buffers(R)
dev = A.device
A.dec_row_map[:R] = 0
A._use_dec_row_map = True
A.state[:R].zero_()
A.state[:R, _lib.TW_ST_LAST:_lib.TW_ST_LASTTS + 1] = -1
A.pos[:R] = 0
A.ids[:R] = st.sot
for k, tok in enumerate(prompt[1:]):
    A.decoder_step(R, with_logits=False, r_enc=1)
    A.ids[:R] = tok
    A.pos[:R] = k + 1
bb["run_score"][:R].view(W, nb).fill_(-1e9)
bb["run_score"][:R].view(W, nb)[:, 0] = 0.0
bb["fin_score"][:R] = -1e9
bb["fin_flag"][:R] = 0
bb["fin_len"][:R] = 0
bb["win"][:W] = torch.tensor([1, 0, 0, 0], dtype=torch.int32, device=dev)
A.state[:R, _lib.TW_ST_NGEN] = 0
sel = A._select_params(0, max_new, True)
bp = _lib.TwBeamParams(nb, max_new, 1.0, A.d.max_target_positions)
bst = _lib.TwBeamState(bb["run_score"].data_ptr(), bb["fin_score"].data_ptr(), bb["fin_flag"].data_ptr(),
                       bb["fin_len"].data_ptr(), bb["fin_tokens"].data_ptr(), bb["win"].data_ptr(),
                       bb["src_rows"].data_ptr())
s = A.stream.cuda_stream
L, H, T = A.d.decoder_layers, A.d.heads, A.d.max_target_positions
for step in range(max_new):
    A.decoder_step(R, r_enc=1)
    torch.cuda.synchronize()
    toks = A.tokens[:R, :step].cpu().numpy()
    lg = A.logits[:R].float().cpu().numpy()
    worst = 0.0
    for r in range(R):
        ref = tf_logits([int(x) for x in toks[r]])
        d = float(np.abs(lg[r] - ref).max())
        worst = max(worst, d)
        if d > 0.05:
            print(f"step {step} row {r}: logits differ by {d:.3f}; history {list(toks[r])}")
    print(f"step {step}: worst row |d| {worst:.4f}", flush=True)
    _lib.call("tw_beam_step", A.logits.data_ptr(), W, A.d.vocab, A.suppress_bits.data_ptr(), ctypes.byref(sel),
              ctypes.byref(bp), ctypes.byref(bst), A.state.data_ptr(), A.tokens.data_ptr(), A.ids.data_ptr(),
              A.pos.data_ptr(), bb["ws"].data_ptr(), s)
    _lib.call("tw_kv_reorder", A.kcache.data_ptr(), A.vcache.data_ptr(), bb["kscr"].data_ptr(), bb["vscr"].data_ptr(),
              L, A.max_rows, H, T, R, bb["src_rows"].data_ptr(), A.pos.data_ptr(), s)
torch.cuda.synchronize()
print("fin scores", bb["fin_score"][:R].cpu().numpy())
print("fin best", bb["fin_tokens"][0, : int(bb["fin_len"][0])].tolist())

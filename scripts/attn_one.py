"""One encoder-attention variant at B=24 windows, S=1500, 20 heads, `reps` launches (for rocprofv3 PMC passes).
    python scripts/attn_one.py VARIANT PAD [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "turbo-whisper-workspace_amd")]
import torch  # noqa: E402

from twamd import _lib  # noqa: E402

_lib.load()
v, pad = int(sys.argv[1]), int(sys.argv[2])
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
B, S, H = 24, 1500, 20
D = H * 64
qkv = (torch.randn(B * S, 3 * D, device="cuda")).to(torch.bfloat16)
qkv[:, :D] = (qkv[:, :D].float() * 0.125).to(torch.bfloat16)
out = torch.empty(B * S, D, dtype=torch.bfloat16, device="cuda")
s = torch.cuda.current_stream().cuda_stream
_lib.call("tw_attn_set_variant", v)
_lib.call("tw_attn_set_lds_pad", pad)
for _ in range(reps):
    _lib.call("tw_attn_encoder", qkv.data_ptr(), B, S, H, out.data_ptr(), s)
torch.cuda.synchronize()
print("ok", v, pad)

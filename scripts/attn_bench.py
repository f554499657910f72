"""A/B timing of the encoder attention kernels at B=24 windows, S=1500, 20 heads (interleaved, one process).
    python scripts/attn_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "turbo-whisper-workspace_amd")]
import torch  # noqa: E402

from twamd import _lib  # noqa: E402

_lib.load()
B, S, H = 24, 1500, 20
D = H * 64
qkv = (torch.randn(B * S, 3 * D, device="cuda")).to(torch.bfloat16)
qkv[:, :D] = (qkv[:, :D].float() * 0.125).to(torch.bfloat16)
out = torch.empty(B * S, D, dtype=torch.bfloat16, device="cuda")
s = torch.cuda.current_stream().cuda_stream
fl = 4.0 * S * S * 64 * H * B
res = {v: [] for v in (8, 10, 12, 14)}
outs = {}
for r in range(5):
    for v in (8, 10, 12, 14):
        _lib.call("tw_attn_set_variant", v)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(5):
            _lib.call("tw_attn_encoder", qkv.data_ptr(), B, S, H, out.data_ptr(), s)
        b.record()
        torch.cuda.synchronize()
        res[v].append(a.elapsed_time(b) / 5)
        if r == 0:
            outs[v] = out.float().clone()
for v, t in res.items():
    print(f"variant {v}: min {min(t):.3f} ms = {fl / min(t) / 1e9:.0f} TF/s  max|diff vs v8| = "
          f"{(outs[v] - outs[8]).abs().max().item():.3g}")
_lib.call("tw_attn_set_variant", 10)

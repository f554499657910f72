"""A/B timing of the encoder attention kernels at B=24 windows, S=1500, 20 heads (interleaved, one process), with
the LDS cap the engine applies beside a running decode (pad 4) and without it (pad 0).
    python scripts/attn_bench.py [--lib path/to/libtwhip.so] [variants...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "turbo-whisper-workspace_amd")]
import torch  # noqa: E402

from twamd import _lib  # noqa: E402

args = sys.argv[1:]
if args[:1] == ["--lib"]:  # another build (A/B across builds)
    _lib.load(args[1])
    args = args[2:]
else:
    _lib.load()
B, S, H = 24, 1500, 20
D = H * 64
VAR = [int(v) for v in args] or [16, 32, 8]
qkv = (torch.randn(B * S, 3 * D, device="cuda")).to(torch.bfloat16)
qkv[:, :D] = (qkv[:, :D].float() * 0.125).to(torch.bfloat16)
out = torch.empty(B * S, D, dtype=torch.bfloat16, device="cuda")
s = torch.cuda.current_stream().cuda_stream
fl = 4.0 * S * S * 64 * H * B
res = {(v, p): [] for v in VAR for p in (0, 4)}
outs = {}
for r in range(5):
    for v in VAR:
        for p in (0, 4):
            _lib.call("tw_attn_set_variant", v)
            _lib.call("tw_attn_set_lds_pad", p)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(5):
                _lib.call("tw_attn_encoder", qkv.data_ptr(), B, S, H, out.data_ptr(), s)
            b.record()
            torch.cuda.synchronize()
            res[(v, p)].append(a.elapsed_time(b) / 5)
            if r == 0 and p == 0:
                outs[v] = out.clone()
_lib.call("tw_attn_set_lds_pad", 0)
for (v, p), t in res.items():
    same = torch.equal(outs[v].view(torch.int16), outs[VAR[0]].view(torch.int16))
    print(f"variant {v} pad {p}: min {min(t):.3f} ms = {fl / min(t) / 1e9:.0f} TF/s  bit-identical to v{VAR[0]}: {same}"
          f"  max|diff| {(outs[v].float() - outs[VAR[0]].float()).abs().max().item():.3g}")
_lib.call("tw_attn_set_variant", 16)

"""Decode-step durations while the encoder runs vs while it is idle, from a rocprofv3 kernel trace.
    python scripts/overlap_stats.py gpurun_out/<tag>"""
import bisect
import csv
import glob
import sys

rows = []
for f in glob.glob(sys.argv[1] + "/kt/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Stream_Id"]))
rows.sort()
ENC = ("k_gemm_big", "k_attn_encoder", "k_layernorm", "k_im2col_conv1", "k_im2col_conv2", "k_logmel")
m = []
for s, e in sorted((s, e) for s, e, n, _ in rows if n in ENC):
    if m and s <= m[-1][1]:
        m[-1][1] = max(m[-1][1], e)
    else:
        m.append([s, e])
starts = [x[0] for x in m]


def active(t):
    i = bisect.bisect_right(starts, t) - 1
    return i >= 0 and m[i][1] >= t


for stream in sorted({st for *_, n, st in rows if n == "k_select_final"}):
    fins = [s for s, e, n, st in rows if n == "k_select_final" and st == stream]
    steps = [(fins[i], fins[i + 1] - fins[i]) for i in range(len(fins) - 1) if fins[i + 1] - fins[i] < 5e6]
    a = [d for t, d in steps if active(t)]
    b = [d for t, d in steps if not active(t)]
    print(f"stream {stream}: decode step with encoder active n={len(a)} avg={sum(a) / max(1, len(a)) / 1e3:.1f}us; "
          f"idle n={len(b)} avg={sum(b) / max(1, len(b)) / 1e3:.1f}us")
print(f"encoder busy {sum(e - s for s, e in m) / 1e6:.1f} ms; trace span {(rows[-1][1] - rows[0][0]) / 1e6:.1f} ms")

"""Per-kernel breakdown of decode steps that run while no encoder kernel is active, from a rocprofv3 kernel trace.
    python scripts/decode_breakdown.py gpurun_out/<tag>"""
import collections
import csv
import glob
import sys

ENC = ("k_gemm_big", "k_gemm_8p", "k_attn_enc2", "k_attn_encoder", "k_layernorm", "k_im2col_conv1", "k_im2col_conv2",
       "k_logmel", "k_logmel_finalize")
rows = []
for f in glob.glob(sys.argv[1] + "/kt/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "")
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, r["Grid_Size_X"], r["Grid_Size_Y"]))
rows.sort()
encs = [(s, e) for s, e, n, *_ in rows if n in ENC]


def busy(s, e):
    return any(not (e2 < s or s2 > e) for s2, e2 in encs)


dec = [r for r in rows if r[2] not in ENC and r[2].startswith("k_")]
steps, cur = [], []
for r in dec:
    cur.append(r)
    if r[2] == "k_select_final":
        steps.append(cur)
        cur = []
n_common = collections.Counter(len(s) for s in steps).most_common(1)[0][0]
idle = [s for s in steps if len(s) == n_common and not busy(s[0][0], s[-1][1])]
act = [s for s in steps if len(s) == n_common and busy(s[0][0], s[-1][1])]
agg = collections.defaultdict(list)
for s in idle:
    for i, r in enumerate(s):
        agg[(i, r[2], r[3], r[4])].append((r[1] - r[0]) / 1e3)
med = lambda v: sorted(v)[len(v) // 2]
tot = 0.0
for k in sorted(agg):
    m = med(agg[k])
    tot += m
    print(f"{k[0]:3d} {k[1]:24s} grid {k[2]:>7s}x{k[3]:<3s} {m:7.2f} us")
span = lambda s: (s[-1][1] - s[0][0]) / 1e3
print(f"{len(steps)} steps, {len(idle)} idle ({n_common} kernels): kernel sum {tot:.1f} us, step span "
      f"{med([span(s) for s in idle]):.1f} us; with encoder active: {len(act)} steps, span "
      f"{med([span(s) for s in act]) if act else 0:.1f} us")

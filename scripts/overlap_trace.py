"""Decode steps that overlap encoder kernels, from a rocprofv3 kernel trace: per-kernel durations (execution,
start->end) and the gaps between consecutive decode kernels (dispatch waits), plus encoder kernel durations
while decode steps run beside them vs alone.
    python scripts/overlap_trace.py gpurun_out/<tag>"""
import collections
import csv
import glob
import sys

ENC = ("k_gemm_big", "k_gemm_8p", "k_gemm_mx", "k_gemm_8p_mx", "k_attn_enc2", "k_attn_encoder", "k_layernorm",
       "k_layernorm_mx", "k_attn_encoder_mx", "k_im2col_conv1", "k_im2col_conv2", "k_logmel", "k_logmel_finalize")
rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "")
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
rows.sort()
encs = [(s, e, n) for s, e, n in rows if n in ENC]
dec = [(s, e, n) for s, e, n in rows if n not in ENC and n.startswith("k_")]


def overlaps(s, e, lst):
    return any(not (e2 < s or s2 > e) for s2, e2, _ in lst)


steps, cur = [], []
for r in dec:
    cur.append(r)
    if r[2] == "k_select_final":
        steps.append(cur)
        cur = []
act = [st for st in steps if overlaps(st[0][0], st[-1][1], encs)]
idle = [st for st in steps if not overlaps(st[0][0], st[-1][1], encs)]
for label, group in (("encoder active", act), ("alone", idle)):
    if not group:
        continue
    execs = sum(sum(e - s for s, e, _ in st) for st in group) / len(group) / 1e3
    span = sum(st[-1][1] - st[0][0] for st in group) / len(group) / 1e3
    per = collections.defaultdict(list)
    for st in group:
        for s, e, n in st:
            per[n].append((e - s) / 1e3)
    print(f"{label}: {len(group)} steps, span {span:.1f} us, kernel exec sum {execs:.1f} us, gaps {span - execs:.1f} us")
    for n, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        print(f"    {n:24s} n/step {len(v) / len(group):5.1f} avg {sum(v) / len(v):8.2f} us")
# encoder kernels: duration when a decode kernel overlaps vs not
ed = collections.defaultdict(lambda: [[], []])
for s, e, n in encs:
    ed[n][1 if overlaps(s, e, dec) else 0].append((e - s) / 1e3)
for n, (a, b) in ed.items():
    f = lambda v: f"{len(v):4d} x {sum(v) / len(v):8.1f} us" if v else "       -"
    print(f"{n:18s} alone {f(a)}   beside decode {f(b)}")

"""Experiment: decode-step kernel time vs dispatch gaps, encoder idle vs active (rocprofv3 kernel trace dir)."""
import collections
import csv
import glob
import sys

ENC = ("k_gemm_big", "k_gemm_8p", "k_gemm_8pp", "k_attn_enc2", "k_attn_encoder", "k_layernorm", "k_im2col_conv1",
       "k_im2col_conv2", "k_logmel", "k_logmel_finalize")
rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "")
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
rows.sort()
encs = [(s, e, n) for s, e, n in rows if n in ENC]


def overlapping(s, e):
    return [n for s2, e2, n in encs if not (e2 < s or s2 > e)]


dec = [r for r in rows if r[2] not in ENC and r[2].startswith("k_")]
steps, cur = [], []
for r in dec:
    cur.append(r)
    if r[2] == "k_select_final":
        steps.append(cur)
        cur = []
n = collections.Counter(len(s) for s in steps).most_common(1)[0][0]
for label, sel in (("idle", lambda s: not overlapping(s[0][0], s[-1][1])), ("active", lambda s: overlapping(s[0][0], s[-1][1]))):
    ss = [s for s in steps if len(s) == n and sel(s)]
    if not ss:
        continue
    k = sum((r[1] - r[0]) for s in ss for r in s) / len(ss) / 1e3
    g = sum((s[i][0] - s[i - 1][1]) for s in ss for i in range(1, len(s))) / len(ss) / 1e3
    print(f"{label}: {len(ss)} steps, kernel time {k:.1f} us/step, gaps {g:.1f} us/step")
# which encoder kernels overlap the biggest gaps
gapby = collections.Counter()
for s in steps:
    for i in range(1, len(s)):
        g0, g1 = s[i - 1][1], s[i][0]
        if g1 - g0 > 20000:
            for nme in set(overlapping(g0, g1)):
                gapby[nme] += (g1 - g0) / 1e3
print("gap time (>20us gaps) by overlapping encoder kernel:", {k: round(v) for k, v in gapby.most_common()})

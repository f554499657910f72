"""Report for coresid.py's trace: per GEMM launch, the small kernels launched beside it (start offset, duration)."""
import csv
import glob
import sys

rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "")
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n, r["Grid_Size_X"]))
rows.sort()
gemms = [r for r in rows if r[2].startswith("k_gemm")]
small = [r for r in rows if r[2] == "k_resid_ln"]
for gs, ge, gn, grid in gemms:
    beside = [r for r in small if gs <= r[0] <= ge + 1]
    print(f"{gn} grid {grid} dur {(ge - gs) / 1e3:.1f} us: {len(beside)} small kernels ran inside; "
          + " ".join(f"{(s - gs) / 1e3:.0f}+{(e - s) / 1e3:.1f}" for s, e, *_ in beside[:12]))

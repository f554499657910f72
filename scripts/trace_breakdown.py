"""Per-(kernel, grid) duration breakdown of a rocprofv3 kernel trace: python scripts/trace_breakdown.py DIR [filter]"""
import collections
import csv
import glob
import sys

d = collections.defaultdict(list)
flt = sys.argv[2] if len(sys.argv) > 2 else ""
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if flt in r["Kernel_Name"]:
            key = (r["Kernel_Name"][:48], int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]), r["Grid_Size_Y"],
                   r["Grid_Size_Z"], r["Workgroup_Size_X"])
            d[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
tot = sum(sum(v) for v in d.values())
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:40]:
    print(f"{str(k):80s} n={len(v):6d} avg={sum(v) / len(v) / 1e3:9.2f}us min={min(v) / 1e3:8.2f} "
          f"tot={sum(v) / 1e6:8.2f}ms {100 * sum(v) / tot:5.1f}%")

"""Per-kernel duration table of a rocprofv3 kernel trace (p50 / mean / count), and the per-call critical-path
view of serial runs: python tools/trace_table.py gpurun_out/TAG/run_kernel_trace.csv"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for r in rows:
    d[r["Kernel_Name"].split("(")[0]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for n, v in sorted(d.items(), key=lambda x: -sorted(x[1])[len(x[1]) // 2]):
    v.sort()
    print(f"{n:40s} n={len(v):5d} p50={v[len(v) // 2]:9.1f} us  mean={sum(v) / len(v):9.1f} us")

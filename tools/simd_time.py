"""SIMD-time share per kernel in a bench's timed window of a rocprofv3 kernel trace: sum over launches of
duration x waves (each stage kernel holds one 512-register wave per SIMD, so wave-time ~ SIMD-time; it
over-counts launches whose waves finish unevenly).  Tooling only.
    python tools/simd_time.py run_kernel_trace.csv bench.json"""
import csv
import json
import sys
from collections import defaultdict

b = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
t0, t1 = b["timed_window_monotonic_ns"]
acc, wall = defaultdict(float), defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s < t0 or e > t1:
        continue
    n = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0]
    waves = (int(r["Grid_Size_X"]) + 63) // 64
    acc[n] += (e - s) * 1e-9 * waves
    wall[n] += (e - s) * 1e-6
tot = sum(acc.values())
win = (t1 - t0) * 1e-9
print(f"window {win * 1e3:.1f} ms, wave-seconds {tot:.2f} = {tot / win / 1024:.2f} x 1024 SIMDs")
for n, v in sorted(acc.items(), key=lambda x: -x[1]):
    print(f"{n:24s} {100 * v / tot:5.1f}%  wave-s {v:7.3f}  busy-ms {wall[n]:8.2f}")

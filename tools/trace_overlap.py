"""Summarise a rocprofv3 kernel trace: per-queue use and the time-weighted number of concurrently running
kernels / waves over the busy span (tools for reading profiles/, not part of the product)."""
import csv
import sys
from collections import Counter

rows = list(csv.DictReader(open(sys.argv[1])))
ev = []
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    waves = (int(r["Grid_Size_X"]) + 63) // 64
    ev.append((s, e, r["Kernel_Name"].split("(")[0], int(r["Queue_Id"]), waves))
ev = [x for x in ev if x[2].startswith("k_") and x[2] != "k_debug_op"]
ev.sort()
print("queues:", Counter(x[3] for x in ev))
pts = sorted([(x[0], 1, x[4]) for x in ev] + [(x[1], -1, -x[4]) for x in ev])
t0, t1 = pts[0][0], pts[-1][0]
cur = cw = 0
last = t0
acc_k = acc_w = 0.0
for t, d, w in pts:
    acc_k += cur * (t - last)
    acc_w += cw * (t - last)
    cur += d
    cw += w
    last = t
span = t1 - t0
print(f"span {span/1e6:.2f} ms, mean concurrent kernels {acc_k/span:.2f}, mean resident waves {acc_w/span:.0f}")
agg = {}
for s, e, n, q, w in ev:
    a = agg.setdefault(n, [0, 0.0])
    a[0] += 1
    a[1] += (e - s) / 1e6
for n, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"{n:20s} {c:5d} launches  avg {t/c:8.3f} ms  total {t:9.2f} ms")

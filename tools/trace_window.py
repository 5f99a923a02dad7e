"""Time-weighted resident waves (capped at the chip's 1,024 SIMDs: one 512-register wave each) and concurrent
kernels over the busiest window of a rocprofv3 kernel trace -- the bench's timed region.  Tooling only.
    python tools/trace_window.py run_kernel_trace.csv [window_ms]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
win = float(sys.argv[2]) * 1e6 if len(sys.argv) > 2 else 500e6
ev = []
for r in rows:
    n = r["Kernel_Name"].split("(")[0].replace("void ", "")
    if not n.startswith("k_") or n.startswith("k_debug"):
        continue
    waves = (int(r["Grid_Size_X"]) + 63) // 64
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n, waves))
ev.sort()
best = None
for s0, _, _, _ in ev:
    busy = sum(max(0, min(e, s0 + win) - max(s, s0)) for s, e, _, _ in ev)
    if best is None or busy > best[0]:
        best = (busy, s0)
s0 = best[1]
s1 = s0 + win
pts = []
for s, e, n, w in ev:
    a, b = max(s, s0), min(e, s1)
    if a < b:
        pts += [(a, 1, w), (b, -1, -w)]
pts.sort()
cur = cw = 0
last = s0
acc_k = acc_w = acc_cap = 0.0
for t, d, w in pts:
    acc_k += cur * (t - last)
    acc_w += cw * (t - last)
    acc_cap += min(cw, 1024) * (t - last)
    cur += d
    cw += w
    last = t
span = s1 - s0
print(f"window {win/1e6:.0f} ms: mean concurrent kernels {acc_k/span:.2f}, mean waves {acc_w/span:.0f}, "
      f"SIMD occupancy (waves capped at 1024) {acc_cap/span/1024:.3f}")

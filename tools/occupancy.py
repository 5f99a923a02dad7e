"""Chip occupancy from a rocprofv3 kernel trace (tools for reading profiles/, not part of the product).

    python tools/occupancy.py run_kernel_trace.csv [--from-ms A --to-ms B] [--json out.json]

Per kernel: launches, total / average duration, waves per launch, the waves per SIMD its registers and LDS allow, and
its SIMD-time = duration x min(SIMDs, waves) / SIMDs (SIMD-equivalents it held; an upper bound, a trace has no tail
shape).  Over the window: the busy span, the time-weighted SIMDs held by all running kernels (capped at the chip's
1,024) = an upper bound of the fraction of SIMDs that had a wave to issue, and the idle fraction (no kernel running).
"""
import argparse
import csv
import json

SIMDS = 1024  # 256 CUs x 4
LDS_PER_CU = 160 * 1024
REGS_PER_LANE = 512  # unified VGPR + AGPR file per SIMD lane (gfx950)


def waves_per_simd(vgpr, agpr, lds, wg):
    regs = ((vgpr + 7) // 8) * 8 + ((agpr + 7) // 8) * 8 if agpr else ((vgpr + 7) // 8) * 8
    wps = min(8, REGS_PER_LANE // max(regs, 8))
    if lds:
        wg_waves = max(1, (wg + 63) // 64)
        wps = min(wps, (LDS_PER_CU // lds) * wg_waves // 4 or 1)
    return max(1, wps)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--from-ms", type=float, default=None)
    ap.add_argument("--to-ms", type=float, default=None)
    ap.add_argument("--json", default=None)
    ap.add_argument("--window", default=None, help="bench.py JSON: keep the kernels inside its timed_window_monotonic_ns")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ev = []
    for r in rows:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if not name.startswith("k_") or name.startswith("k_debug"):
            continue
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        wg = int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"])
        waves = (grid + 63) // 64
        wps = waves_per_simd(int(r["VGPR_Count"]), int(r["Accum_VGPR_Count"]), int(r["LDS_Block_Size"]), wg)
        ev.append((s, e, name, waves, wps))
    ev.sort()
    if a.window:
        line = [l for l in open(a.window) if l.startswith("{")][-1]
        w0, w1 = json.loads(line)["timed_window_monotonic_ns"]
        ev = [x for x in ev if x[0] >= w0 and x[1] <= w1]
    t0 = ev[0][0]
    if a.from_ms is not None:
        ev = [x for x in ev if (x[0] - t0) / 1e6 >= a.from_ms]
    if a.to_ms is not None:
        ev = [x for x in ev if (x[1] - t0) / 1e6 <= a.to_ms]
    pts = sorted([(s, 1, min(SIMDS, w)) for s, e, n, w, p in ev] + [(e, -1, -min(SIMDS, w)) for s, e, n, w, p in ev])
    w0, w1 = pts[0][0], pts[-1][0]
    held = 0
    cur = 0
    last = w0
    acc_held = 0.0
    idle = 0.0
    for t, d, simds in pts:
        dt = t - last
        acc_held += min(SIMDS, held) * dt
        if cur == 0:
            idle += dt
        cur += d
        held += simds
        last = t
    span = w1 - w0
    agg = {}
    for s, e, n, w, p in ev:
        g = agg.setdefault(n, {"launches": 0, "ms": 0.0, "waves": 0, "wps": p, "simd_ms": 0.0})
        g["launches"] += 1
        g["ms"] += (e - s) / 1e6
        g["waves"] += w
        g["simd_ms"] += (e - s) / 1e6 * min(SIMDS, w) / SIMDS
    total_simd = sum(g["simd_ms"] for g in agg.values())
    out = {"span_ms": round(span / 1e6, 3), "idle_frac": round(idle / span, 4),
           "simd_held_frac_upper": round(acc_held / (SIMDS * span), 4),
           "kernels": {n: {"launches": g["launches"], "total_ms": round(g["ms"], 3),
                           "avg_ms": round(g["ms"] / g["launches"], 4),
                           "avg_waves": round(g["waves"] / g["launches"], 1), "waves_per_simd_cap": g["wps"],
                           "simd_ms": round(g["simd_ms"], 3),
                           "simd_share": round(g["simd_ms"] / total_simd, 4) if total_simd else 0}
                       for n, g in sorted(agg.items(), key=lambda x: -x[1]["simd_ms"])}}
    print(f"span {out['span_ms']} ms  idle {out['idle_frac']:.3f}  SIMDs held (upper bound) {out['simd_held_frac_upper']:.3f}")
    print(f"{'kernel':28s} {'n':>5s} {'avg ms':>9s} {'avg waves':>10s} {'w/SIMD':>6s} {'SIMD-ms':>9s} {'share':>6s}")
    for n, k in out["kernels"].items():
        print(f"{n:28s} {k['launches']:5d} {k['avg_ms']:9.3f} {k['avg_waves']:10.1f} {k['waves_per_simd_cap']:6d} "
              f"{k['simd_ms']:9.2f} {k['simd_share']:6.3f}")
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()

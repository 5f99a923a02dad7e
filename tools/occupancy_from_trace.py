"""How full the chip is during the timed window of a kernel trace (rocprofv3 --kernel-trace CSV of bench.py): at every
instant, the waves the running dispatches could keep resident (a dispatch's waves, capped by what its register
allocation lets the 1,024 SIMDs hold: 1 per SIMD at > 256 VGPR+AGPR, 2 at <= 256, ...), summed over concurrent
dispatches and capped at the chip's 1,024 SIMDs x that kernel's waves per SIMD -- reported as the time-average SIMD
fill (1.0 = every SIMD holding work every instant), the idle fraction (no dispatch running) and the fill per phase.
Tooling only.

    python tools/occupancy_from_trace.py run_kernel_trace.csv bench.json
"""
import csv
import json
import sys

SIMDS = 1024


def waves_per_simd(vgpr, agpr):
    regs = ((vgpr + 7) // 8) * 8 + ((agpr + 7) // 8) * 8
    for lim, w in ((64, 8), (72, 7), (80, 6), (96, 5), (128, 4), (168, 3), (256, 2)):
        if regs <= lim:
            return w
    return 1


def main(trace, bench_json):
    lines = open(bench_json).read().strip().splitlines()
    b = json.loads(lines[-1])
    t0, t1 = b["timed_window_monotonic_ns"]
    ev = []
    per_kernel = {}
    for r in csv.DictReader(open(trace)):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if e <= t0 or s >= t1:
            continue
        s, e = max(s, t0), min(e, t1)
        wg = int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"])
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        waves = max(1, (grid + 63) // 64) if wg else 1
        wps = waves_per_simd(int(r["VGPR_Count"]), int(r["Accum_VGPR_Count"]))
        simd_share = min(1.0, waves / (SIMDS * wps))  # the fraction of the SIMDs' wave slots this dispatch can use
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0]
        ev.append((s, simd_share))
        ev.append((e, -simd_share))
        k = per_kernel.setdefault(name, [0, 0.0, 0.0])
        k[0] += 1
        k[1] += (e - s) * 1e-6
        k[2] += (e - s) * 1e-6 * simd_share
    ev.sort()
    fill_t = idle_t = 0.0
    cur, last = 0.0, t0
    for t, d in ev:
        dt = t - last
        fill_t += min(1.0, cur) * dt
        if cur <= 1e-9:
            idle_t += dt
        cur += d
        last = t
    dt = t1 - last
    fill_t += min(1.0, max(cur, 0.0)) * dt
    if cur <= 1e-9:
        idle_t += dt
    win = t1 - t0
    out = {"window_ms": win * 1e-6, "mean_simd_fill": round(fill_t / win, 4), "idle_fraction": round(idle_t / win, 4),
           "kernels": {k: {"dispatches": v[0], "busy_ms": round(v[1], 3), "simd_ms": round(v[2], 3)}
                       for k, v in sorted(per_kernel.items(), key=lambda kv: -kv[1][2])}}
    return out


if __name__ == "__main__":
    o = main(sys.argv[1], sys.argv[2])
    print(f"window {o['window_ms']:.1f} ms  mean SIMD fill {o['mean_simd_fill']:.3f}  idle {o['idle_fraction']:.3f}")
    for k, v in list(o["kernels"].items())[:14]:
        print(f"  {k:26s} {v['dispatches']:4d}  busy {v['busy_ms']:8.2f} ms  SIMD-ms {v['simd_ms']:8.2f}")
    if len(sys.argv) > 3:
        json.dump(o, open(sys.argv[3], "w"), indent=1)

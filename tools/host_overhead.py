#!/usr/bin/env python3
"""Where an isolated call's latency goes: wall time of ctx.verify_raw against the device time the runtime reports
(blsgpu_stats.device_ms: first kernel of the run to its results on the host), per config, nothing else in flight.

    python tools/host_overhead.py [--configs C2,C1,C5] [--reps 7] [--out gpurun_out/host_overhead.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C2,C1,C5")
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import bench
    from lodestar_amd.native import Context

    ctx = Context([0])
    rows = []
    for cfg in a.configs.split(","):
        work, n_sets, desc, _ = bench.build_workload(ctx, cfg, 0)
        work.pop("expected", None)
        call = {k: v for k, v in bench.message_variant(ctx, work, 0).items() if not k.startswith("_")}
        ctx.verify_raw(**call, seed=bench.SEED)  # warm
        wall, dev = [], []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            _, st = ctx.verify_raw(**call, seed=bench.SEED)
            wall.append((time.perf_counter() - t0) * 1e3)
            dev.append(st.device_ms)
        row = {"config": cfg, "sets": n_sets, "wall_p50_ms": round(float(np.median(wall)), 3),
               "device_p50_ms": round(float(np.median(dev)), 3),
               "host_p50_ms": round(float(np.median(np.array(wall) - np.array(dev))), 3)}
        print(json.dumps(row), flush=True)
        rows.append(row)
    if a.out:
        json.dump({"tool": "tools/host_overhead.py", "rows": rows}, open(a.out, "w"), indent=1)
    ctx.close()


if __name__ == "__main__":
    main()

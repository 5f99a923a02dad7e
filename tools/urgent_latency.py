#!/usr/bin/env python3
"""Isolated latency of urgent calls (BLSGPU_JOB_URGENT: the reference's verifyOnMainThread, one job of 1 or 3 single
sets, table mode) -- nothing else in flight.  For a kernel trace of the lane's critical path:

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/T -- python3 tools/urgent_latency.py --reps 10
    python tools/trace_call.py gpurun_out/T/.../*kernel_trace.csv 2

    python tools/urgent_latency.py [--reps 20] [--set urgent_cus=8 ...] [--out FILE]
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
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import bench
    from lodestar_amd.native import Context

    ctx = Context([0])
    for kv in args.set:
        k, _, v = kv.partition("=")
        ctx.set_option(k, int(v))
    work, _, _, _ = bench.build_workload(ctx, "C1", 0)
    calls = bench.urgent_calls(ctx, work)
    lat = []
    for i in range(4 + 2 * args.reps):
        n, kw = calls[i % len(calls)]
        t1 = time.perf_counter()
        res, st = ctx.verify_raw(**kw, seed=bench.URGENT_SEED)
        assert res[0] == 1 and st.urgent_lane == 1
        if i >= 4:  # the first calls build the lane's buffers
            lat.append((n, (time.perf_counter() - t1) * 1e3, 1))
    out = {"isolated_ms": bench.urgent_summary(lat), "options": {k: ctx.get_option(k) for k in
                                                                 ("urgent_cus", "urgent_isolate", "urgent_excl")}}
    print(json.dumps(out), flush=True)
    if args.out:
        with open(args.out, "w") as fh:
            json.dump(out, fh)
    ctx.close()


if __name__ == "__main__":
    main()

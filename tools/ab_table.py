"""Summarises interleaved A/B bench lines (tools/gpurun/r06_f.sh and earlier A/B scripts): per variant, value / hash-stage frac /
isolated stage times / p50.   python tools/ab_table.py gpurun_out/TAG"""
import glob
import json
import statistics
import sys
from collections import defaultdict

rows = defaultdict(list)
for f in sorted(glob.glob(sys.argv[1] + "_*_*.json")):
    lines = [l for l in open(f) if l.startswith("{")]
    if not lines:
        continue
    d = json.loads(lines[-1])
    var = f[len(sys.argv[1]) + 1:].rsplit("_", 1)[0]
    rows[var].append(d)
for var, ds in rows.items():
    v = [d["value"] for d in ds]
    iso = {k: round(statistics.mean(d["roofline"]["isolated_call"][k]["ms"] for d in ds), 2)
           for k in ds[0]["roofline"]["isolated_call"]}
    st = {k: round(statistics.mean(d["roofline"]["stages"][k]["tproducts_per_s"] for d in ds), 2)
          for k in ds[0]["roofline"]["stages"]}
    print(f"{var:24s} n={len(v)} value={[round(x / 1e6, 3) for x in v]} mean={statistics.mean(v) / 1e6:.3f}M "
          f"frac={statistics.mean(d['roofline']['frac'] for d in ds):.3f} "
          f"pipe={statistics.mean(d['roofline']['pipeline_frac'] for d in ds):.3f} "
          f"p50={statistics.mean(d['p50_batch_latency_ms'] for d in ds):.1f}ms")
    print("   isolated ms", iso)
    print("   stage Tprod/s", st)

"""Isolated-call latency and per-stage isolated times of bench lines: python tools/lat_table.py FILE..."""
import json
import sys

for f in sys.argv[1:]:
    lines = [l for l in open(f) if l.startswith("{")]
    if not lines:
        print(f, "no line")
        continue
    d = json.loads(lines[-1])
    iso = d.get("roofline", {}).get("isolated_call", {})
    print(f"{f}: value {d['value']:.0f} p50 {d['p50_batch_latency_ms']} ms | " +
          " ".join(f"{k}={v['ms']:.2f}" for k, v in iso.items()))

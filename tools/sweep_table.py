"""Prints the bench lines of a gpurun sweep log (tools/gpurun/sweep.sh) as a table."""
import json
import sys

cur = None
for line in open(sys.argv[1]):
    if line.startswith("=="):
        cur = line.strip()[3:]
        continue
    try:
        d = json.loads(line)
    except ValueError:
        continue
    r = d.get("roofline", {})
    st = {k: v["ms_per_launch"] for k, v in r.get("stages", {}).items()}
    print(f"{cur:60s} {d['value']:12.0f} frac {r.get('pipeline_frac', 0):.3f} p50 {d.get('p50_batch_latency_ms')} "
          f"miller {st.get('miller_sets')} check {st.get('group_check')}")

"""Summary of an A/B run of a round-4 isolation A/B script (git history: tools/gpurun/r04_iso_ab.sh): per variant, the isolation-profile stage table
(tools/iso_table.py) and the 20-step C2 bench value.  Tooling only.
    python tools/ab_iso_report.py TAG SETS variant ..."""
import contextlib
import io
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import iso_table  # noqa: E402

tag, sets, variants = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
for v in variants:
    print(f"=== {v}")
    p = f"gpurun_out/{tag}_{v}_iso/run_kernel_stats.csv"
    if os.path.exists(p):
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            iso_table.main(p, sets)
        for line in buf.getvalue().splitlines():
            if not line.startswith("   ") or any(k in line for k in ("hash_map", "hash_clear", "miller", "decode", "finish")):
                print(line)
    else:
        print("  (no isolation profile)")
    j = f"gpurun_out/{tag}_{v}_c2.json"
    try:
        d = json.loads([l for l in open(j) if l.startswith("{")][-1])
        print(f"  C2 {d['value']:.0f} sets/s, p50 {d['p50_batch_latency_ms']} ms")
    except Exception:
        print("  (no C2 bench)")

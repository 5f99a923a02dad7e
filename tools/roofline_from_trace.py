"""Recomputes bench.py's `roofline` for the dominant stage from a committed rocprofv3 kernel trace of the same
command: the launches of the stage's kernels that fall inside the bench's timed window
(`timed_window_monotonic_ns`, CLOCK_MONOTONIC like rocprofv3's timestamps), grouped into pipeline runs, each run's
stage interval (first kernel start -> last kernel end, as the bench's HIP events bracket it) and its summed kernel
durations; frac = algorithmic products per launch / interval / peak.  Tooling only (no GPU).

    python tools/roofline_from_trace.py gpurun_out/r03e_prof/run_kernel_trace.csv gpurun_out/r03e_prof.json \
        [profiles/r03_roofline_check.json]
"""
import csv
import json
import sys


def main(trace, bench_json, out=None):
    line = [l for l in open(bench_json) if l.startswith("{")][-1]
    b = json.loads(line)
    rf = b["roofline"]
    names = rf["kernel"].split("+")
    t0, t1 = b["timed_window_monotonic_ns"]
    ev = []
    for r in csv.DictReader(open(trace)):
        n = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0]
        if n not in names:
            continue
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s >= t0 and e <= t1:
            ev.append((s, e, n, int(r["Grid_Size_X"]), r.get("Queue_Id", "0")))
    ev.sort()
    # a run's stage starts at its k_hash_prep (names[0]) and holds the stage kernels that follow it on the same
    # queue up to that queue's next k_hash_prep (consecutive runs alternate between stream pairs and overlap in
    # time, so grouping by time alone would hand one run's tail to the next)
    runs, cur = [], {}
    for s, e, n, g, q in ev:
        if n == names[0]:
            cur[q] = {"start": s, "end": e, "kernel_ns": 0, "kernels": 0, "prep_grid": g}
            runs.append(cur[q])
        if q not in cur:
            continue
        c = cur[q]
        c["end"] = max(c["end"], e)
        c["kernel_ns"] += e - s
        c["kernels"] += 1
        if n == names[-1]:
            c["complete"] = True
    # only runs whose last kernel (names[-1]) landed inside the window (the stage lists alternative forms, e.g. the
    # lane-pair and cooperative clearings, so a run launches fewer kernels than the list names)
    done = [r for r in runs if r.get("complete")]
    span = sum(r["end"] - r["start"] for r in done) / len(done) / 1e6
    busy = sum(r["kernel_ns"] for r in done) / len(done) / 1e6
    prods = rf["algorithmic_products_per_launch"] * rf["launches_timed"] / max(len(done), 1)
    doc = {
        "source": {"trace": trace, "bench": bench_json},
        "stage_kernels": names,
        "runs_in_window": len(done),
        "bench_launches_timed": rf["launches_timed"],
        "trace_interval_ms_per_launch": round(span, 4),
        "trace_kernel_busy_ms_per_launch": round(busy, 4),
        "bench_avg_launch_ms": rf["avg_launch_ms"],
        "algorithmic_products_per_launch": prods,
        "frac_from_trace_interval": round(prods / (span * 1e-3) / (rf["peak"] * 1e12), 4),
        "frac_bench": rf["frac"],
    }
    doc["agreement"] = round(doc["frac_from_trace_interval"] / rf["frac"], 3)
    s = json.dumps(doc, indent=1)
    print(s)
    if out:
        open(out, "w").write(s + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:])

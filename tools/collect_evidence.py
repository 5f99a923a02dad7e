"""Folds one round-end evidence call (tools/gpurun/r06_h.sh TAG: GPU suite + smoke, then r06_final.sh TAGf with its
driver-command profile TAGfe) from gpurun_out/ into the committed profiles/ files the DESIGN tables cite, and prints
the table rows.  Host-only tooling.

    python tools/collect_evidence.py TAG [ROUND]        (ROUND default r06)

Writes profiles/ROUND_bench_final_{C2,C2_100,C1,C3,C4,C5,host8,urgent}.json (each bench.py line as printed),
ROUND_curve_final.json, ROUND_driver_kernel_{trace,stats}.csv, ROUND_pmc_traffic.json (already written on the box by
r06_final.sh; copied back so the committed file carries the shipped library's md5), ROUND_sq_counters.json,
ROUND_roofline_check.json, ROUND_gpu_tests_final.log, ROUND_urgent_kernel_trace_summary.json is left to
tools/urgent_wait.py.
"""
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PROF = os.path.join(ROOT, "profiles")


def last_json(path):
    return json.loads([l for l in open(path) if l.startswith("{")][-1])


def main():
    tag = sys.argv[1]
    rnd = sys.argv[2] if len(sys.argv) > 2 else "r06"
    f, fe = tag + "f", tag + "fe"
    rows = []
    for cfg in ["C2", "C2_100", "C1", "C3", "C4", "C5", "host8", "urgent"]:
        src = os.path.join(OUT, f"{f}_{cfg}.json")
        if not os.path.exists(src):
            print("missing", src)
            continue
        d = last_json(src)
        json.dump(d, open(os.path.join(PROF, f"{rnd}_bench_final_{cfg}.json"), "w"), indent=1)
        r = d.get("roofline") or {}
        par = d.get("parity") if isinstance(d.get("parity"), dict) else {}
        cb = d.get("cpu_baseline") or {}
        rows.append((cfg, round(d["value"]), d.get("ms_per_step"), d.get("p50_batch_latency_ms"),
                     d.get("call_latency_under_load_ms"), r.get("frac"), r.get("pipeline_frac"),
                     par.get("jobs"), par.get("mismatches"), cb.get("value"), (cb.get("all_cores") or {}).get("value")))
    curve = os.path.join(OUT, f"{f}_curve.json")
    if os.path.exists(curve):
        shutil.copy(curve, os.path.join(PROF, f"{rnd}_curve_final.json"))
    tr = os.path.join(OUT, f"{fe}_trace")
    for name in ["kernel_trace", "kernel_stats"]:
        p = os.path.join(tr, f"run_{name}.csv")
        if os.path.exists(p):
            shutil.copy(p, os.path.join(PROF, f"{rnd}_driver_{name}.csv"))
    pmc = os.path.join(OUT, f"{f}_pmc_traffic.json")
    if os.path.exists(pmc):
        shutil.copy(pmc, os.path.join(PROF, f"{rnd}_pmc_traffic.json"))
    sq = os.path.join(OUT, f"{fe}_sq1", "run_counter_collection.csv")
    if os.path.exists(sq):
        subprocess.run([sys.executable, os.path.join(ROOT, "tools", "sq_to_json.py"), sq,
                        os.path.join(PROF, f"{rnd}_sq_counters.json"), os.path.join(tr, "run_kernel_trace.csv"),
                        os.path.join(OUT, f"{fe}_trace.json")], check=True, stdout=subprocess.DEVNULL)
    if os.path.exists(os.path.join(tr, "run_kernel_trace.csv")):
        subprocess.run([sys.executable, os.path.join(ROOT, "tools", "roofline_from_trace.py"),
                        os.path.join(tr, "run_kernel_trace.csv"), os.path.join(OUT, f"{fe}_trace.json"),
                        os.path.join(PROF, f"{rnd}_roofline_check.json")], check=True, stdout=subprocess.DEVNULL)
    log = os.path.join(OUT, f"{tag}_gpu_tests.log")
    if os.path.exists(log):
        shutil.copy(log, os.path.join(PROF, f"{rnd}_gpu_tests_final.log"))
    print("cfg sets/s ms/step p50_iso under_load frac pipeline_frac parity_jobs mismatches cpu16 cpu_all")
    for r in rows:
        print(*r)


if __name__ == "__main__":
    main()

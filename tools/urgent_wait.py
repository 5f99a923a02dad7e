#!/usr/bin/env python3
"""Where urgent-lane kernels wait under load, from a rocprofv3 kernel trace of
`bench.py --urgent-every-ms X` (the isolated urgent calls run first, alone, so the queues that carry kernels before the
first gossip call's kernels are the urgent lane's queues).

Per urgent-lane kernel name: launches, mean / max execution time, and mean / max "queue gap" = its start minus the end
of the previous kernel on the same queue (the lane's kernels of one branch follow each other on one queue, so a gap is
time the kernel waited for free SIMDs or for a cross-branch event).  Split into the isolated phase and the loaded one.

    python tools/urgent_wait.py gpurun_out/TAG/run_kernel_trace.csv [--json out.json]
"""
import csv
import json
import sys
from collections import defaultdict


def main(path, out=None):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    name = lambda r: r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0]
    # the first kernel of a gossip run: a hash_prep whose grid covers a 16k call's messages
    first_big = next(i for i, r in enumerate(rows) if name(r) == "k_hash_prep" and int(r["Grid_Size_X"]) >= 16384)
    uq = {r["Queue_Id"] for r in rows[:first_big] if not name(r).startswith("__amd")}
    t_load = int(rows[first_big]["Start_Timestamp"])
    # (the warm-up and signing kernels before the isolated urgent calls run on other queues / the table stream: the
    # urgent queues are those of k_miller_coop / k_group_check launches before the flood)
    uq = {r["Queue_Id"] for r in rows[:first_big] if name(r) in ("k_miller_coop", "k_group_check", "k_hash_clear_coop",
                                                                  "k_group_sig_miller", "k_sig_subgroup_coop")}
    prev_end = {}
    stats = {"isolated": defaultdict(list), "loaded": defaultdict(list)}
    for r in rows:
        q = r["Queue_Id"]
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if q in uq and not name(r).startswith("__amd"):
            gap = (s - prev_end[q]) / 1e3 if q in prev_end else None
            phase = "loaded" if s >= t_load else "isolated"
            stats[phase][name(r)].append(((e - s) / 1e3, gap))
        if q in uq:
            prev_end[q] = e
    res = {"urgent_queues": sorted(uq), "phases": {}}
    for ph, d in stats.items():
        res["phases"][ph] = {}
        for k, v in sorted(d.items(), key=lambda kv: -sum(x[0] for x in kv[1])):
            ex = [x[0] for x in v]
            gp = [x[1] for x in v if x[1] is not None and x[1] < 200000]
            res["phases"][ph][k] = {"n": len(v), "exec_us_mean": round(sum(ex) / len(ex), 1), "exec_us_max": round(max(ex), 1),
                                    "gap_us_mean": round(sum(gp) / len(gp), 1) if gp else None,
                                    "gap_us_max": round(max(gp), 1) if gp else None}
    print(json.dumps(res, indent=1))
    if out:
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[3] if len(sys.argv) > 3 and sys.argv[2] == "--json" else None)

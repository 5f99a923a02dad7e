#!/usr/bin/env python3
"""Where urgent-lane kernels wait under load, from a rocprofv3 kernel trace of
`bench.py --urgent-every-ms X` (the urgent lane's queues are those that ran the cooperative small-run kernels; an urgent
kernel is "loaded" when a pipeline kernel ran during it, "isolated" otherwise).

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
    # the urgent lane's queues: those that ran the cooperative small-run kernels (a C2 flood run never does)
    coop = ("k_miller_coop", "k_hash_clear_coop", "k_sig_subgroup_coop")
    uq = {r["Queue_Id"] for r in rows if name(r) in coop}
    # intervals of pipeline (non-urgent) kernels, merged, to tell a loaded urgent kernel from an isolated one
    busy = []
    for r in rows:
        if r["Queue_Id"] in uq or name(r).startswith("__amd"):
            continue
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if busy and s <= busy[-1][1]:
            busy[-1][1] = max(busy[-1][1], e)
        else:
            busy.append([s, e])
    import bisect

    starts = [b[0] for b in busy]

    def loaded(s, e):
        k = bisect.bisect_right(starts, e) - 1
        return k >= 0 and busy[k][1] >= s

    prev_end = {}
    stats = {"isolated": defaultdict(list), "loaded": defaultdict(list)}
    for r in rows:
        q = r["Queue_Id"]
        if q not in uq:
            continue
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if not name(r).startswith("__amd"):
            gap = (s - prev_end[q]) / 1e3 if q in prev_end else None
            stats["loaded" if loaded(s, e) else "isolated"][name(r)].append(((e - s) / 1e3, gap))
        prev_end[q] = e
    res = {"urgent_queues": sorted(uq), "phases": {}}
    for ph, d in stats.items():
        res["phases"][ph] = {}
        for k, v in sorted(d.items(), key=lambda kv: -sum(x[0] for x in kv[1])):
            ex = [x[0] for x in v]
            gp = [x[1] for x in v if x[1] is not None and x[1] < 5000]  # gaps inside a call (< 5 ms)
            res["phases"][ph][k] = {"n": len(v), "exec_us_mean": round(sum(ex) / len(ex), 1),
                                    "exec_us_max": round(max(ex), 1),
                                    "gap_us_mean": round(sum(gp) / len(gp), 1) if gp else None}
    print(json.dumps(res, indent=1))
    if out:
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[3] if len(sys.argv) > 3 and sys.argv[2] == "--json" else None)

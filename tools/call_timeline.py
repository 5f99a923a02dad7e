#!/usr/bin/env python3
"""Kernel timeline of the LAST verification call in a rocprofv3 kernel trace (the call starts at its k_hash_prep,
minus a few kernels before it on other queues): start / end (ms from the call's first kernel), duration, queue, grid.

    python tools/call_timeline.py gpurun_out/TAG/run_kernel_trace.csv
"""
import csv
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "k_hash_prep" in r["Kernel_Name"]]
    last = [r for r in rows[idx[-1] - 3:] if "rocclr" not in r["Kernel_Name"] or True]
    t0 = int(last[0]["Start_Timestamp"])
    for r in last:
        s = (int(r["Start_Timestamp"]) - t0) / 1e6
        e = (int(r["End_Timestamp"]) - t0) / 1e6
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        print(f"{name[:34]:34} q{r['Queue_Id']:>2} {s:8.3f} {e:8.3f} {e - s:7.3f}  grid {r['Grid_Size_X']:>7} wg {r['Workgroup_Size_X']}")


if __name__ == "__main__":
    main(sys.argv[1])

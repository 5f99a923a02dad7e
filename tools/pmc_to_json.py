"""Folds the two rocprofv3 PMC passes of tools/gpurun/pmc.sh (FETCH_SIZE, WRITE_SIZE; csv output) into
profiles/<tag>_pmc_traffic.json: per kernel, the counter summed over each dispatch's rows and averaged over
dispatches (kB per launch, as rocprofv3 reports them).  bench.py turns them into HBM bytes per launch.

    python tools/pmc_to_json.py gpurun_out/r01_pmc2 profiles/r01_pmc_traffic.json
"""
import csv
import json
import sys
from collections import defaultdict


def per_launch(path, counter):
    """kernel -> (kB per launch, launches, bytes per grid work-item)"""
    per_dispatch = defaultdict(float)
    names, grid = {}, {}
    with open(path) as fh:
        for row in csv.DictReader(fh):
            if row["Counter_Name"] != counter:
                continue
            per_dispatch[row["Dispatch_Id"]] += float(row["Counter_Value"])
            names[row["Dispatch_Id"]] = row["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0]
            grid[row["Dispatch_Id"]] = int(row["Grid_Size"])
    acc = defaultdict(list)
    items = defaultdict(int)
    for d, v in per_dispatch.items():
        acc[names[d]].append(v)
        items[names[d]] += grid[d]
    return {k: (sum(v) / len(v), len(v), 1024 * sum(v) / max(items[k], 1)) for k, v in acc.items()}


def lib_md5(path=None):
    """md5 of the libblsgpu.so the passes measured (the same file travels to the GPU box): bench.py flags its
    `traffic` as stale when the library it loads differs."""
    import hashlib
    import os

    path = path or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lodestar_amd",
                                "libblsgpu.so")
    with open(path, "rb") as fh:
        return hashlib.md5(fh.read()).hexdigest()


def main(prefix, out):
    f = per_launch(f"{prefix}_pmc_FETCH_SIZE/run_counter_collection.csv", "FETCH_SIZE")
    w = per_launch(f"{prefix}_pmc_WRITE_SIZE/run_counter_collection.csv", "WRITE_SIZE")
    kernels = {k: {"FETCH_SIZE_kB_per_launch": round(f.get(k, (0, 0, 0))[0], 1),
                   "WRITE_SIZE_kB_per_launch": round(w.get(k, (0, 0, 0))[0], 1),
                   "launches": f.get(k, (0, 0, 0))[1],
                   # launch sizes differ (merged runs): bytes per grid work-item, the launch-size-independent figure
                   "FETCH_B_per_item": round(2 * f.get(k, (0, 0, 0))[2], 1),
                   "WRITE_B_per_item": round(w.get(k, (0, 0, 0))[2], 1)} for k in sorted(set(f) | set(w))}
    doc = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes, kernel trace only), "
                     "bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-parity --no-profile (the driver command; C2, merged runs)",
           "units": "kB per launch as reported; gfx950 FETCH_SIZE counts 1/2 of wide streaming reads "
                    "(MI355X_MICROARCH.md HBM section) -> bytes = 2 x 1024 x FETCH_SIZE; WRITE_SIZE exact. "
                    "*_B_per_item: HBM bytes per grid work-item over all dispatches (FETCH already doubled)",
           "lib_md5": lib_md5(),
           "kernels": kernels}
    with open(out, "w") as fh:
        json.dump(doc, fh, indent=1)
    return doc


if __name__ == "__main__":
    d = main(sys.argv[1], sys.argv[2])
    for k, v in d["kernels"].items():
        print(k, v)

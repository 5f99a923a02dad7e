"""Folds a rocprofv3 SQ/GRBM PMC pass of the driver's command (tools/gpurun/evidence.sh) into a per-kernel VALU table:

  * wave_cycles        SQ_WAVE_CYCLES summed over the kernel's dispatches (wave-resident cycles, per XCD sums added)
  * frac_active_valu   SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES: the fraction of a resident wave's cycles in which it was
                       issuing VALU work (the VALU-utilisation the north star asks for; 1 wave/SIMD kernels: the SIMD's)
  * frac_wait_any      SQ_WAIT_ANY / SQ_WAVE_CYCLES (waiting on memory / dependencies)
  * valu_insts_per_wave, waves
and, with a kernel trace of the same command (optional) and lodestar_amd/op_counts.json, the achieved
v_mad_u64_u32 rate of the stage kernels: Montgomery products of the launch x 392 MADs / average launch time.

    python tools/sq_to_json.py gpurun_out/r4x_sq1/run_counter_collection.csv profiles/r04_sq_counters.json \
        [kernel_trace.csv bench.json]
"""
import csv
import json
import sys
from collections import defaultdict

COUNTERS = ["SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
            "SQ_ACTIVE_INST_VALU", "SQ_INSTS_VALU", "GRBM_GUI_ACTIVE", "GRBM_COUNT"]


def short(name):
    return name.split("(")[0].replace("void ", "").split("<")[0]


def main(path, out):
    per = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for r in csv.DictReader(open(path)):
        c = r["Counter_Name"]
        if c not in COUNTERS:
            continue
        k = short(r["Kernel_Name"])
        per[k][c] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    kernels = {}
    for k, v in per.items():
        wc = v["SQ_WAVE_CYCLES"] or 1.0
        kernels[k] = {
            "dispatches": len(disp[k]),
            "waves": v["SQ_WAVES"],
            "wave_cycles": v["SQ_WAVE_CYCLES"],
            "frac_active_valu": round(v["SQ_ACTIVE_INST_VALU"] / wc, 4),
            "frac_active_any": round(v["SQ_ACTIVE_INST_ANY"] / wc, 4),
            "frac_wait_any": round(v["SQ_WAIT_ANY"] / wc, 4),
            "frac_wait_inst_any": round(v["SQ_WAIT_INST_ANY"] / wc, 4),
            "valu_insts_per_wave": round(v["SQ_INSTS_VALU"] / max(v["SQ_WAVES"], 1.0), 1),
            "gui_active_cycles": v["GRBM_GUI_ACTIVE"],
        }
    # workload generation (signing on the GPU before timing, the pubkey table fill) is not part of the verified path
    setup = {"k_debug_op", "k_pk_table_fill", "k_signing_roots"}
    for k in setup & set(kernels):
        kernels[k]["setup_not_timed"] = True
    path_k = {k: v for k, v in kernels.items() if k not in setup}
    tot_wc = sum(v["wave_cycles"] for v in path_k.values()) or 1.0
    for v in path_k.values():
        v["share_of_wave_cycles"] = round(v["wave_cycles"] / tot_wc, 4)
    doc = {"source": "rocprofv3 --pmc " + " ".join(COUNTERS) + " (one pass, kernel trace only) over the driver's "
                     "command: bench.py --gpus 1 --steps 20 --warmup 5 (C2, merged runs); per kernel, summed over "
                     "dispatches",
           "weighted_frac_active_valu": round(sum(v["frac_active_valu"] * v["wave_cycles"] for v in path_k.values())
                                              / tot_wc, 4),
           "note": "SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES: the fraction of a resident wave's cycles spent issuing VALU "
                   "(per wave, not per SIMD). The one-lane stage kernels hold one 512-register wave per SIMD, so theirs "
                   "is the SIMD's; the lane-pair and two-wave kernels (k_hash_clear2, k_sig_subgroup2, k_hash_map, "
                   "k_sig_decode, k_msm_bucket2, k_miller_lines2) share a SIMD with a second "
                   "wave, so a wave waits while its partner issues (counted in SQ_WAIT_INST_ANY) and the SIMD's VALU "
                   "share is up to twice the per-wave figure. One wave alone issues a plain VALU instruction every ~4 "
                   "cycles and a v_mad_u64_u32 every ~10 (profiles/r02_mad_chain.json) -- half the SIMD's rate with "
                   "two waves.",
           "kernels": dict(sorted(kernels.items(), key=lambda kv: -kv[1]["wave_cycles"]))}
    with open(out, "w") as fh:
        json.dump(doc, fh, indent=1)
    return doc


if __name__ == "__main__":
    d = main(sys.argv[1], sys.argv[2])
    print("weighted VALU-active fraction", d["weighted_frac_active_valu"])
    for k, v in list(d["kernels"].items())[:16]:
        print(f"{k:24s} share {v.get('share_of_wave_cycles', 0):.3f} valu {v['frac_active_valu']:.3f} "
              f"wait {v['frac_wait_any']:.3f} insts/wave {v['valu_insts_per_wave']:.0f}")

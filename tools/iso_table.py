"""Per-kernel efficiency in an isolation profile (round-4 script in git history, tools/gpurun/r04_iso.sh: one C2 call of N sets per step, every
branch on one stream, so each kernel runs alone on the chip): average launch time, the stage's algorithmic
Montgomery multiplications (lodestar_amd/op_counts.json) and the fraction of the chip's measured Montgomery-product
rate (29.17e12 v_mad_u64_u32 lane-ops/s / 392 MADs per 14-limb product = 7.44e10 products/s).  Tooling only.

    python tools/iso_table.py gpurun_out/r4b_iso/run_kernel_stats.csv 131072 [miller_k]
"""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PEAK = 2.9171e13 / 392
ops = json.load(open(os.path.join(ROOT, "lodestar_amd", "op_counts.json")))


def main(path, n, k=2):
    ps = ops["per_set"]
    groups = max(1, n // 1024)
    stage = {  # kernel-name prefixes -> Montgomery multiplications per launch
        "sig_decode": (["k_sig_decode"], ps["sig_decode"]["total"] * n),
        "hash_to_g2": (["k_hash_prep", "k_hash_map", "k_hash_clear", "k_h_affine", "k_batch_inv"],
                       ps["hash_to_g2"]["total"] * n),
        "pk_finish": (["k_pk_finish", "k_pk_affine"], ps["pk_finish"]["total"] * n),
        "sig_msm": (["k_msm_bucket", "k_msm_slice_pairs", "k_msm_window", "k_msm_horner"],
                    ps["sig_msm"]["total"] * n + ops["per_group_fixed"]["sig_msm"] * groups),
        "miller_lines": (["k_miller_lines", "k_miller_lines2"], ops["miller_lines_per_message"] * n),
        "miller_acc": (["k_miller_acc", "k_miller_acc2"], ops["miller_acc_per_chunk"][str(k)] * n / k),
    }
    rows = {}
    for r in csv.DictReader(open(path)):
        name = r["Name"].split("(")[0].replace("void ", "").split("<")[0]
        rows[name] = (int(r["Calls"]), float(r["AverageNs"]) * 1e-6)
    if "k_miller_acc2" in rows:  # one item per chunk (two lanes per pairing): priced as k = 1
        stage["miller_acc"] = (stage["miller_acc"][0], ops["miller_acc_per_chunk"]["1"] * n)
    calls = rows.get("k_sig_decode", (1, 0))[0]
    tot_ms = 0
    print(f"{'stage / kernel':28s} {'ms/launch':>10s} {'mults/launch':>13s} {'frac':>6s}")
    for st, (kern, mults) in stage.items():
        ms = 0
        for kn in kern:
            c, a = rows.get(kn, (0, 0))
            ms += a * c / calls  # per call (batch_inv runs several times per call)
        tot_ms += ms
        frac = mults / (ms * 1e-3) / PEAK if ms else 0
        print(f"{st:28s} {ms:10.3f} {mults:13.3e} {frac:6.3f}")
        for kn in kern:
            c, a = rows.get(kn, (0, 0))
            print(f"   {kn:25s} {a * c / calls:10.3f}")
    other = sum(a * c / calls for kn, (c, a) in rows.items()
                if not any(kn in v[0] for v in stage.values()) and kn.startswith("k_") and kn != "k_debug_op"
                and kn != "k_pk_table_fill")
    print(f"{'other (groups, F tree, mask)':28s} {other:10.3f}")
    tot = sum(v[1] for v in stage.values())
    print(f"total {tot_ms + other:.2f} ms/call for {n} sets: {n / ((tot_ms + other) * 1e-3):.0f} sets/s serial, "
          f"frac {tot / ((tot_ms + other) * 1e-3) / PEAK:.3f}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]) if len(sys.argv) > 3 else 2)

#!/usr/bin/env python3
"""Checks tools/microbench/limb_forms output: every form's result equals the mad64 form's (the binary counts the
mismatches), and the sampled lanes' results equal x0 * y^ITERS mod p by Python big integers.

    tools/microbench/limb_forms > out.json && python3 tools/microbench/limb_forms_check.py out.json
"""
import json
import sys

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB


def main(path):
    d = json.load(open(path))
    bad = [k for k in ("f64_mismatches",) if d[k]]
    for s in d["samples"]:
        want = int(s["x0"], 16) * pow(int(s["y"], 16), d["iters"], P) % P
        for k in ("x", "x_f64"):
            if int(s[k], 16) != want:
                bad.append(f"sample {s['x0'][:12]} {k}: got {s[k][:12]} want {want:096x}"[:80])
    # the 24-bit integer forms are known wrong on gfx950 (see the .hip header): reported, not gating
    print(f"u24 mismatches {d['u24_mismatches']}, mad64/24 mismatches {d['mad64_24_mismatches']} of {d['lanes_checked']}")
    for r in d["results"]:
        print(f"{r['form']:55s} {r['waves_per_simd']} {r['mont_products_per_s']:.3e}")
    if bad:
        raise SystemExit(f"FAILED: {bad}")
    print(f"ok: mad64 and f64 agree on {d['lanes_checked']} lanes, {len(d['samples'])} samples = x0 y^{d['iters']} mod p")


if __name__ == "__main__":
    main(sys.argv[1])

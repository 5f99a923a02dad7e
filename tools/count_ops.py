#!/usr/bin/env python3
"""Counts the Montgomery multiplications (mul, sqr) each pipeline stage of the device algorithm
performs, by running the host build of the same source (tests/native/emu.cpp, -DBLS_COUNT_OPS).
Writes lodestar_amd/op_counts.json, the algorithmic-work table bench.py's roofline uses.

Unit of algorithmic work: one 32x32->64-bit limb product.  A 381-bit Montgomery multiplication
(or squaring) is priced at 2 * 12^2 = 288 products -- the schoolbook CIOS/FIPS cost with 12 x 32-bit
limbs, independent of this implementation's own 14 x 28-bit layout (which issues 392 / 301 mads).
Run:  python3 tools/count_ops.py
"""
import ctypes
import json
import os
import random
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import bls12_381 as bls  # noqa: E402  (test/tooling use only: builds inputs)
from tests.emu_helpers import f12b, g1b, g2b  # noqa: E402

PRODUCTS_PER_MUL = 288
SO = "/tmp/libbls_emu_count.so"


def main():
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-DBLS_COUNT_OPS", "-o", SO,
                           os.path.join(ROOT, "tests", "native", "emu.cpp")])
    L = ctypes.CDLL(SO)
    L.emu_count_mul.restype = ctypes.c_ulonglong
    L.emu_count_sqr.restype = ctypes.c_ulonglong
    L.emu_stage_sig_scale_w.argtypes = [ctypes.c_char_p, ctypes.c_uint64]
    L.emu_stage_sig_msm.argtypes = [ctypes.c_char_p, ctypes.c_int]
    L.emu_stage_pk_finish_w.argtypes = [ctypes.c_char_p, ctypes.c_uint64]
    L.emu_stage_miller_acc.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int]
    L.emu_g1_mul_u64.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p]
    L.emu_sig_decode.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]

    def measure(fn, reps=1):
        L.emu_count_reset()
        for _ in range(reps):
            fn()
        return (L.emu_count_mul() / reps, L.emu_count_sqr() / reps)

    rnd = random.Random(5)
    msgs = [bytes([i]) * 32 for i in range(8)]
    sig = bls.sign(12345, msgs[0])
    comp = bls.g2_compress(sig)
    pk = bls.sk_to_pk(777)
    out = ctypes.create_string_buffer(576)
    inf = ctypes.c_int()
    scal = [rnd.getrandbits(64) | (1 << 63) for _ in range(16)]
    stages = {}
    stages["sig_decode"] = measure(lambda: L.emu_sig_decode(comp, 96, out, ctypes.byref(inf)))
    m = iter(msgs * 4)
    stages["hash_to_g2"] = measure(lambda: L.emu_hash_to_g2(next(m), out), reps=8)
    s = iter(scal * 2)
    stages["pk_finish"] = measure(lambda: L.emu_stage_pk_finish_w(g1b(pk), next(s)), reps=16)
    s = iter(scal * 2)
    stages["sig_scale"] = measure(lambda: L.emu_stage_sig_scale_w(g2b(sig), next(s)), reps=16)
    # bucket MSM (k_msm.hip): a + b n for a range of n sets -> per set b, per range a
    pts = b"".join(g2b(bls.g2_mul(sig, rnd.randrange(1, bls.R))) for _ in range(256))
    m0 = measure(lambda: L.emu_stage_sig_msm(pts, 0))
    m256 = measure(lambda: L.emu_stage_sig_msm(pts, 256))
    stages["sig_msm"] = ((m256[0] - m0[0]) / 256, (m256[1] - m0[1]) / 256)
    H = bls.hash_to_g2(msgs[1])
    lines = measure(lambda: L.emu_stage_miller_lines(g2b(H)))
    acc = {k: measure(lambda: L.emu_stage_miller_acc(g1b(pk), g2b(H), k)) for k in (1, 2, 4, 8)}
    # per-group stages as a function of group size n: a + b n
    g0 = measure(lambda: L.emu_stage_group_sig_miller(g2b(sig), 0))
    g64 = measure(lambda: L.emu_stage_group_sig_miller(g2b(sig), 64))
    f = bls.miller_loop(pk, H)
    f0 = measure(lambda: L.emu_stage_group_finish(f12b(f), 0))
    f64 = measure(lambda: L.emu_stage_group_finish(f12b(f), 64))
    a0 = measure(lambda: L.emu_stage_pk_aggregate(g1b(pk), 0))
    a512 = measure(lambda: L.emu_stage_pk_aggregate(g1b(pk), 512))
    tot = lambda ms: ms[0] + ms[1]
    res = {
        "products_per_mul": PRODUCTS_PER_MUL,
        "note": "Montgomery multiplications (mul+sqr) of the device algorithm per unit; products = count * 288",
        "per_set": {k: {"mul": v[0], "sqr": v[1], "total": tot(v)} for k, v in stages.items()},
        "per_group_fixed": {"group_sig_miller": tot(g0), "group_finish": tot(f0), "sig_msm": tot(m0)},
        "per_group_per_set": {"group_sig_miller": (tot(g64) - tot(g0)) / 64, "group_finish": (tot(f64) - tot(f0)) / 64},
        "pk_aggregate_per_pubkey": (tot(a512) - tot(a0)) / 512,
        # Miller stage split as the kernels run it: lines once per distinct message, accumulation per chunk of
        # k pairings (shared squarings); per set = lines + acc_chunk[k] / k for distinct messages
        "miller_lines_per_message": tot(lines),
        "miller_acc_per_chunk": {str(k): tot(v) for k, v in acc.items()},
    }
    res["per_set"]["miller_sets"] = {"mul": None, "sqr": None,
                                     "total": tot(lines) + tot(acc[2]) / 2, "note": "lines + acc_chunk[2] / 2"}
    # the pipeline's signature side is the MSM; sig_scale (per-set scaling) is kept for reference only
    per_set_total = sum(v["total"] for k, v in res["per_set"].items() if k != "sig_scale")  # miller_k = 2
    res["per_single_set_total"] = per_set_total
    path = os.path.join(ROOT, "lodestar_amd", "op_counts.json")
    with open(path, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()

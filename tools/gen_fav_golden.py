#!/usr/bin/env python3
"""Generates tests/golden/fav_cases.json: FastAggregateVerify / eth_fast_aggregate_verify / KeyValidate cases
in the shape of the consensus spec tests the reference runs (packages/beacon-node/test/spec/general/bls.ts;
the vectors themselves are not vendored), computed by the KAT-pinned oracle (oracle/bls12_381.py).  Data only.

    python tools/gen_fav_golden.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import bls12_381 as bls  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "fav_cases.json")


def main():
    sks = [int.from_bytes(bytes([0x40 + i]) * 32, "big") % bls.R for i in range(4)]
    pks = [bls.g1_compress(bls.sk_to_pk(s)) for s in sks]
    msg = bytes([0xAB]) * 32
    agg_sk = sum(sks[:3]) % bls.R
    sig3 = bls.g2_compress(bls.sign(agg_sk, msg))
    sig_other = bls.g2_compress(bls.sign(agg_sk, bytes(32)))
    # a curve point outside G1 and a non-curve x (first hits of a fixed scan)
    not_in_group = not_on_curve = None
    for t in range(1, 400):
        cand = bytes([0x80]) + bytes(45) + t.to_bytes(2, "big")
        try:
            pt = bls.g1_decompress(cand)
            if bls.g1_mul(pt, bls.R) is not None and not_in_group is None:
                not_in_group = cand
        except bls.BlstError as e:
            if e.code == bls.BLST_POINT_NOT_ON_CURVE and not_on_curve is None:
                not_on_curve = cand
        if not_in_group and not_on_curve:
            break
    cases = [
        ("valid_3_keys", pks[:3], msg, sig3),
        ("wrong_message", pks[:3], bytes(32), sig3),
        ("signature_over_other_message", pks[:3], msg, sig_other),
        ("missing_key", pks[:2], msg, sig3),
        ("extra_key", pks[:4], msg, sig3),
        ("key_not_in_group", pks[:2] + [not_in_group], msg, sig3),
        ("key_not_on_curve", pks[:2] + [not_on_curve], msg, sig3),
        ("key_infinity", pks[:3] + [bls.G1_INFINITY_COMPRESSED], msg, sig3),
        ("no_keys_infinity_sig", [], msg, bls.G2_INFINITY_COMPRESSED),
        ("no_keys_valid_sig", [], msg, sig3),
        ("signature_bad_encoding", pks[:3], msg, bytes([0x00]) + sig3[1:]),
        ("signature_infinity", pks[:3], msg, bls.G2_INFINITY_COMPRESSED),
        ("single_key", pks[:1], msg, bls.g2_compress(bls.sign(sks[0], msg))),
    ]
    out = {"generator": "tools/gen_fav_golden.py (oracle/bls12_381.py)", "cases": []}
    for name, keys, m, sig in cases:
        out["cases"].append({
            "name": name, "pubkeys": [k.hex() for k in keys], "message": m.hex(), "signature": sig.hex(),
            "fast_aggregate_verify": bls.fast_aggregate_verify(keys, m, sig),
            "eth_fast_aggregate_verify": bls.eth_fast_aggregate_verify(keys, m, sig),
            "key_validate": [(lambda k: 0 if _ok(k) else _code(k))(k) for k in keys],
        })
    with open(OUT, "w") as fh:
        json.dump(out, fh, indent=1)
    print(f"wrote {OUT}: {len(out['cases'])} cases")


def _ok(k):
    try:
        bls.key_validate(k)
        return True
    except bls.BlstError:
        return False


def _code(k):
    try:
        bls.key_validate(k)
        return 0
    except bls.BlstError as e:
        return e.code


if __name__ == "__main__":
    main()

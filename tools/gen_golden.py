#!/usr/bin/env python3
"""Generates tests/golden/verify_sets.json with the CPU oracle (oracle/bls12_381.py, itself pinned by the
reference's KATs in tests/test_oracle_kat.py).  The fixture is data only: keys, signature sets, per-job
expected results for several job layouts, hash_to_G2 outputs and aggregated pubkeys.

Keys and messages follow the reference's own multithread test (packages/beacon-node/test/e2e/chain/bls/
multithread.test.ts:28-41): sk_i = msg_i = (i+1) repeated 32 bytes.  Expected per-job results follow the
reference semantics (SURVEY.md 8a parity contract): 1 valid, 0 well-formed but invalid, -code rejected
(pubkeys are aggregated first, utils.ts:11; then every signature is deserialized, maybeBatch.ts:23,36).

    python tools/gen_golden.py            # rewrites tests/golden/verify_sets.json
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import bls12_381 as bls  # noqa: E402

N_KEYS = 10
OUT = os.path.join(ROOT, "tests", "golden", "verify_sets.json")


def sk_of(i):
    return int.from_bytes(bytes([i + 1]) * 32, "big") % bls.R


def msg_of(i):
    return bytes([i + 1]) * 32


def adversarial():
    """Signatures of every deserialization error class (first candidates found by a fixed scan)."""
    out = {}
    for t in range(1, 200):
        cand = bytes([0x80]) + bytes(46) + bytes([t]) + bytes(48)
        c = bls.classify_signature(cand)
        if c and c not in out:
            out[c] = cand
        if bls.BLST_POINT_NOT_ON_CURVE in out and bls.BLST_POINT_NOT_IN_GROUP in out:
            break
    return out


def expected_job(sets, keys):
    """Reference result of one verifySignatureSets job over `sets` (dicts of this fixture)."""
    if not sets:
        return -10  # "Empty signature set" (maybeBatch.ts:29-31)
    for s in sets:
        if not s["pks"]:
            return -9  # EMPTY_AGGREGATE_ARRAY (utils.ts:11 -> PublicKey.aggregate([]))
    for s in sets:
        c = bls.classify_signature(bytes.fromhex(s["sig"]))
        if c:
            return -c
    tri = [(bls.aggregate_pubkeys([keys[i] for i in s["pks"]]), bytes.fromhex(s["msg"]), bytes.fromhex(s["sig"]))
           for s in sets]
    return int(bls.verify_signature_sets_maybe_batch(tri))


def main():
    sks = [sk_of(i) for i in range(N_KEYS)]
    keys = [bls.sk_to_pk(s) for s in sks]
    sets = []

    def add(name, pks, msg, sig):
        sets.append({"name": name, "pks": pks, "msg": msg.hex(), "sig": sig.hex()})

    for i in range(8):
        add(f"single{i}", [i], msg_of(i), bls.g2_compress(bls.sign(sks[i], msg_of(i))))
    add("wrong_message", [0], msg_of(1), bytes.fromhex(sets[0]["sig"]))
    add("invalid_size_32", [2], msg_of(2), bytes(32))  # multithread.test.ts:89-106
    add("infinity", [3], msg_of(3), bytes([0xC0]) + bytes(95))
    add("bad_encoding_flags", [4], msg_of(4), bytes([0xE0]) + bytes(95))
    adv = adversarial()
    add("not_on_curve", [5], msg_of(5), adv[bls.BLST_POINT_NOT_ON_CURVE])
    add("not_in_group", [6], msg_of(6), adv[bls.BLST_POINT_NOT_IN_GROUP])
    add("uncompressed_192", [3], msg_of(3), bls.g2_serialize(bls.sign(sks[3], msg_of(3))))
    m_agg = bytes(range(32))
    add("aggregate6", [0, 1, 2, 3, 4, 5], m_agg, bls.g2_compress(bls.sign(sum(sks[:6]) % bls.R, m_agg)))
    m_agg2 = bytes(range(32, 64))
    add("aggregate_dup", [6, 7, 3, 3, 9], m_agg2,
        bls.g2_compress(bls.sign((sks[6] + sks[7] + 2 * sks[3] + sks[9]) % bls.R, m_agg2)))
    add("aggregate_missing_signer", [0, 1, 2, 8], m_agg, bls.g2_compress(bls.sign(sum(sks[:3]) % bls.R, m_agg)))
    add("aggregate_empty", [], m_agg, bytes.fromhex(sets[15]["sig"]))
    n = len(sets)
    by = {s["name"]: k for k, s in enumerate(sets)}

    layouts = {
        "each_alone": [[k] for k in range(n)],
        "multi_set_jobs": [[0, 1, 2, 3], [4, 5, by["wrong_message"]], [6, 7, by["uncompressed_192"]],
                           [by["aggregate6"], by["aggregate_dup"]], [by["aggregate_missing_signer"], 0],
                           [by["invalid_size_32"], 1], [], [by["aggregate_empty"], 2], [by["infinity"], 5],
                           [by["not_in_group"], by["not_on_curve"]]],
    }
    cases = []
    for lname, jobs in layouts.items():
        exp = [expected_job([sets[k] for k in j], keys) for j in jobs]
        for batchable in (False, True):
            cases.append({"name": f"{lname}/{'batchable' if batchable else 'plain'}", "jobs": jobs,
                          "batchable": batchable, "expected": exp})

    h2g = [{"msg": m.hex(), "g2": bls.g2_serialize(bls.hash_to_g2(m)).hex()}
           for m in [msg_of(i) for i in range(4)] + [b"", b"abc", m_agg]]
    aggs = [{"pks": s["pks"], "pk": bls.g1_serialize(bls.aggregate_pubkeys([keys[i] for i in s["pks"]])).hex()}
            for s in sets if len(s["pks"]) > 1]
    doc = {
        "generator": "tools/gen_golden.py (oracle/bls12_381.py)",
        "keys_source": "sk_i = (i+1) repeated 32 bytes (reference multithread.test.ts:28-41)",
        "keys": [{"sk": f"{sks[i]:064x}", "pk": bls.g1_serialize(keys[i]).hex()} for i in range(N_KEYS)],
        "sets": sets,
        "cases": cases,
        "hash_to_g2": h2g,
        "aggregate_pubkeys": aggs,
    }
    with open(OUT, "w") as f:
        json.dump(doc, f, indent=1)
    print(f"wrote {OUT}: {n} sets, {len(cases)} cases")


if __name__ == "__main__":
    main()

"""Pins the C restatement (oracle/blscpu.c, the large-size oracle and cpu_baseline) against the reference's
known-answer data and the KAT-pinned Python oracle, on the committed golden fixture."""
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

from oracle import bls12_381 as bls
from oracle import cpu, ssz_min

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
FX = json.load(open(os.path.join(GOLDEN, "verify_sets.json")))

DEPOSIT_PK = bytes.fromhex("a99a76ed7796f7be22d5b7e85deeb7c5677e88e511e0b337618f8c4eb61349b4bf2d153f649f7b53359fe8b94a38e44c")
DEPOSIT_SIG = bytes.fromhex(
    "a95af8ff0f8c06af4d29aef05ce865f85f82df42b606008ec5b1bcb42b17ae47f4b78cdce1db31ce32d18f42a6b296b4"
    "014a2164981780e56b5a40d7723c27b8423173e58fa36f075078b177634f66351412b867c103f532aedd50bcd9b98446")
DEPOSIT_ROOT = bytes.fromhex("f9e9adcff9c1517685beae7922ba8d8743626199d2bd7b397f3bd97ac140b542")
CACHED_PKS = [
    "8be678633e927aa0435addad5dcd5283fef6110d91362519cd6d43e61f6c017d724fa579cc4b2972134e050b6ba120c0",
    "8e602f8ec17777c22f465f9b4707c2840647790f15f5c33bd8850f274d5c320850105639960ae4effe57aa5dd279bb98",
    "832a777fe5d89724583bcce5b4794d0b38be419a2daed09d7ee6af2c7c09465e0e2cd07a305c38e59e83e211e8ded246",
    "8076b9d469d71902e06cce3af0528c190850d3dabfb8314eba1ef4eb789131de0dd75d2fe4b7964f347bfe61597cde54",
]
CACHED_SKS = [
    0x0E5BD52621B6A8956086DCF0ECC89F0CDCA56CEBB2A8516C2D4252A9867FC551,
    0x19773A731561958A4F257B85AF81769BCB1146476936C4D9ADD796D4D3FDA020,
    0x6C9E69A6781538C945EAD231AECBEC9CF6CA3500DF59BC85F711FC97A768694E,
    0x2948F046357E74993187A6EF40ACB961911C52AC7A4257BABE6AF197F447E892,
]


def test_deposit_kat():
    """reference beacon-node/test/e2e/interop/genesisState.test.ts:51-55: sign byte-equal, verify true."""
    sk = bls.interop_secret_key(0).to_bytes(32, "big")
    pk96 = cpu.sk_to_pk(sk)
    st, pk_from_48 = cpu.pk_decode(DEPOSIT_PK)
    assert st == 0 and pk_from_48 == pk96
    assert cpu.key_validate(DEPOSIT_PK) == 0
    assert cpu.sign(sk, DEPOSIT_ROOT) == DEPOSIT_SIG
    res, _ = cpu.verify_jobs(job_first_set=[0, 1, 2], sigs=DEPOSIT_SIG * 2, sig_len=[96, 96],
                             msgs=DEPOSIT_ROOT + bytes(32), pk_bytes=pk96 * 2, job_flags=[0, 0])
    assert list(res) == [1, 0]


def test_cached_keys_kat():
    """reference cli/test/utils/cachedKeys.ts:15-26: sk -> compressed pk byte-equal, KeyValidate ok."""
    pks = cpu.sk_to_pk(b"".join(s.to_bytes(32, "big") for s in CACHED_SKS))
    for i, h in enumerate(CACHED_PKS):
        st, dec = cpu.pk_decode(bytes.fromhex(h))
        assert st == 0 and dec == pks[96 * i: 96 * i + 96]
        assert cpu.key_validate(bytes.fromhex(h)) == 0
        assert cpu.key_validate(dec) == 0


def test_mainnet_g2_points_and_infinity():
    pts = json.load(open(os.path.join(GOLDEN, "mainnet_g2_points.json")))["points"]
    for h in pts:
        assert cpu.sig_status(bytes.fromhex(h)) == 0
    assert cpu.sig_status(bytes([0xC0]) + bytes(95)) == 0  # constants.test.ts:5-9 decodes (to infinity)
    assert cpu.sig_status(bytes(32)) == bls.BLST_INVALID_SIZE  # multithread.test.ts:100


def test_hash_to_g2_golden():
    for h in FX["hash_to_g2"]:
        m = bytes.fromhex(h["msg"])
        if len(m) == 32:
            assert cpu.hash_to_g2(m).hex() == h["g2"]


def test_signature_error_classes_match_python_oracle():
    for s in FX["sets"]:
        sig = bytes.fromhex(s["sig"])
        assert cpu.sig_status(sig) == bls.classify_signature(sig), s["name"]


def test_keys_and_signatures_match_python_oracle():
    for k in FX["keys"]:
        assert cpu.sk_to_pk(bytes.fromhex(k["sk"])).hex() == k["pk"]
    for s in FX["sets"]:
        if s["name"].startswith("single") and len(s["pks"]) == 1:
            sk = bytes.fromhex(FX["keys"][s["pks"][0]]["sk"])
            m = bytes.fromhex(s["msg"])
            assert cpu.sign(sk, m) == bls.g2_compress(bls.sign(int.from_bytes(sk, "big"), m))


def _flatten(jobs):
    jfs, order = [0], []
    for j in jobs:
        order += j
        jfs.append(len(order))
    return jfs, [FX["sets"][k] for k in order]


@pytest.mark.parametrize("case", [c["name"] for c in FX["cases"]])
@pytest.mark.parametrize("mode", ["table", "bytes_aggregate"])
def test_golden_cases(case, mode):
    c = next(x for x in FX["cases"] if x["name"] == case)
    jfs, sets = _flatten(c["jobs"])
    sigs = [bytes.fromhex(s["sig"]) for s in sets]
    spf, idx = [0], []
    for s in sets:
        idx += s["pks"]
        spf.append(len(idx))
    keys = b"".join(bytes.fromhex(k["pk"]) for k in FX["keys"])
    common = dict(job_first_set=jfs, sigs=b"".join(x.ljust(192, b"\0")[:192] for x in sigs),
                  sig_len=[len(x) for x in sigs], msgs=b"".join(bytes.fromhex(s["msg"]) for s in sets),
                  set_pk_first=spf, job_flags=[int(c["batchable"])] * len(c["jobs"]), sig_stride=192)
    if mode == "table":
        table = cpu.Table(keys)
        res, _ = cpu.verify_jobs(table=table, pk_index=idx, **common)
    else:
        res, _ = cpu.verify_jobs(pk_bytes=b"".join(keys[96 * i: 96 * i + 96] for i in idx), **common)
    assert list(res) == c["expected"]


def test_aggregate_pubkeys_golden():
    keys = b"".join(bytes.fromhex(k["pk"]) for k in FX["keys"])
    spf, idx = [0], []
    for a in FX["aggregate_pubkeys"]:
        idx += a["pks"]
        spf.append(len(idx))
    n = len(FX["aggregate_pubkeys"])
    out, st = cpu.aggregate_pubkeys(table=cpu.Table(keys), job_first_set=[0, n], sigs=bytes(96 * n),
                                    sig_len=[96] * n, msgs=bytes(32 * n), set_pk_first=spf, pk_index=idx)
    assert (st == 0).all()
    assert [o.hex() for o in out] == [a["pk"] for a in FX["aggregate_pubkeys"]]
    out48, _ = cpu.aggregate_pubkeys(table=cpu.Table(keys), out_len=48, job_first_set=[0, n], sigs=bytes(96 * n),
                                     sig_len=[96] * n, msgs=bytes(32 * n), set_pk_first=spf, pk_index=idx)
    for o, a in zip(out48, FX["aggregate_pubkeys"]):
        pt = bls.g1_deserialize(bytes.fromhex(a["pk"]))
        assert o == bls.g1_compress(pt)


def test_key_validate_classes():
    """KeyValidate (processDeposit.ts:56-64 PublicKey.fromBytes(pk, validate=true)): infinity, bad flags,
    x >= p, not on curve, not in G1."""
    assert cpu.key_validate(bytes([0xC0]) + bytes(47)) == bls.BLST_PK_IS_INFINITY
    assert cpu.key_validate(bytes([0x40]) + bytes(95)) == bls.BLST_PK_IS_INFINITY
    assert cpu.key_validate(bytes(48)) == bls.BLST_BAD_ENCODING  # compressed flag missing
    assert cpu.key_validate(bytes([0x9F]) + bytes([0xFF]) * 47) == bls.BLST_BAD_ENCODING  # x >= p
    assert cpu.key_validate(bytes(47)) == bls.BLST_INVALID_SIZE
    seen = set()
    for t in range(1, 600):
        cand = bytes([0x80]) + bytes(45) + t.to_bytes(2, "big")
        want = None
        try:
            pt = bls.g1_decompress(cand)
            want = 0 if bls.g1_mul(pt, bls.R) is None else bls.BLST_POINT_NOT_IN_GROUP
        except bls.BlstError as e:
            want = e.code
        assert cpu.key_validate(cand) == want
        seen.add(want)
    assert {bls.BLST_POINT_NOT_ON_CURVE, bls.BLST_POINT_NOT_IN_GROUP} <= seen


def test_random_batches_match_python_oracle():
    """Random jobs (valid, wrong-message, swapped-signature) through the pool restatement vs the Python
    maybe-batch restatement."""
    rng = np.random.default_rng(7)
    n = 24
    sks = [bls.interop_secret_key(i) for i in range(n)]
    msgs = [hashlib.sha256(bytes([i])).digest() for i in range(n)]
    sigs = bytearray(cpu.sign(b"".join(s.to_bytes(32, "big") for s in sks), b"".join(msgs)))
    pks = cpu.sk_to_pk(b"".join(s.to_bytes(32, "big") for s in sks))
    sigs[96 * 3: 96 * 4] = sigs[96 * 4: 96 * 5]  # set 3 carries set 4's signature
    msgs[9] = hashlib.sha256(b"other").digest()  # set 9 signed another message
    sizes = [int(x) for x in rng.integers(1, 4, 12)]
    jfs = np.concatenate([[0], np.cumsum(sizes)])
    jfs = jfs[jfs <= n]
    if jfs[-1] != n:
        jfs = np.append(jfs, n)
    for flags in (1, 0):
        res, st = cpu.verify_jobs(job_first_set=jfs, sigs=bytes(sigs), sig_len=[96] * n, msgs=b"".join(msgs),
                                  pk_bytes=pks, job_flags=[flags] * (len(jfs) - 1))
        want = []
        for j in range(len(jfs) - 1):
            sets = [(bls.g1_deserialize(pks[96 * i: 96 * i + 96]), msgs[i], bytes(sigs[96 * i: 96 * i + 96]))
                    for i in range(jfs[j], jfs[j + 1])]
            want.append(int(bls.verify_signature_sets_maybe_batch(sets)))
        assert list(res) == want
        assert want.count(0) >= 1


@pytest.mark.slow
def test_sanitizer_selftest():
    """ASan + UBSan build of the oracle restatement and its self-test (sanitizers on host code)."""
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "sanitize"], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "selftest ok" in r.stdout

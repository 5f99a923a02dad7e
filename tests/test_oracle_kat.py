"""Pins the CPU oracle against the reference's own known-answer data."""
import json
import os
import random

import pytest

from oracle import bls12_381 as bls
from oracle import ssz_min

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_curve_constants():
    z = bls.BLS_X
    assert bls.R == z**4 - z**2 + 1
    assert bls.P == ((z - 1) ** 2 * bls.R) // 3 + z
    assert bls.on_curve(bls.Fp1Ops, bls.G1_GEN)
    assert bls.on_curve(bls.Fp2Ops, bls.G2_GEN)
    assert bls.g1_mul(bls.G1_GEN, bls.R) is None
    assert bls.g2_mul(bls.G2_GEN, bls.R) is None
    assert 3 * (bls.P**4 - bls.P**2 + 1) // bls.R == (z - 1) ** 2 * (z + bls.P) * (z**2 + bls.P**2 - 1) + 3


def test_interop_deposit_kat():
    """reference packages/beacon-node/test/e2e/interop/genesisState.test.ts:51-55 (minimal preset)."""
    pk = bytes.fromhex("a99a76ed7796f7be22d5b7e85deeb7c5677e88e511e0b337618f8c4eb61349b4bf2d153f649f7b53359fe8b94a38e44c")
    wc = bytes.fromhex("00fad2a6bfb0e7f1f0f45460944fbd8dfa7f37da06a4d13b3983cc90bb46963b")
    sig = bytes.fromhex(
        "a95af8ff0f8c06af4d29aef05ce865f85f82df42b606008ec5b1bcb42b17ae47f4b78cdce1db31ce32d18f42a6b296b4"
        "014a2164981780e56b5a40d7723c27b8423173e58fa36f075078b177634f66351412b867c103f532aedd50bcd9b98446"
    )
    sk = bls.interop_secret_key(0)
    assert sk == 0x25295F0D1D592A90B333E26E85149708208E9F8E8BC18F6C77BD62F8AD7A6866
    assert bls.g1_compress(bls.sk_to_pk(sk)) == pk
    root = ssz_min.compute_signing_root(
        ssz_min.deposit_message_root(pk, wc, 32_000_000_000),
        ssz_min.compute_domain(ssz_min.DOMAIN_DEPOSIT, bytes.fromhex("00000001")),
    )
    assert root.hex() == "f9e9adcff9c1517685beae7922ba8d8743626199d2bd7b397f3bd97ac140b542"
    assert bls.g2_compress(bls.sign(sk, root)) == sig
    assert bls.core_verify(bls.g1_decompress(pk), root, bls.signature_from_bytes(sig))
    assert not bls.core_verify(bls.g1_decompress(pk), bytes(32), bls.signature_from_bytes(sig))


def test_cached_keys_kat():
    """reference packages/cli/test/utils/cachedKeys.ts:15-26 (sk = KeyGen(0xaa+i repeated))."""
    pks = [
        "8be678633e927aa0435addad5dcd5283fef6110d91362519cd6d43e61f6c017d724fa579cc4b2972134e050b6ba120c0",
        "8e602f8ec17777c22f465f9b4707c2840647790f15f5c33bd8850f274d5c320850105639960ae4effe57aa5dd279bb98",
        "832a777fe5d89724583bcce5b4794d0b38be419a2daed09d7ee6af2c7c09465e0e2cd07a305c38e59e83e211e8ded246",
        "8076b9d469d71902e06cce3af0528c190850d3dabfb8314eba1ef4eb789131de0dd75d2fe4b7964f347bfe61597cde54",
    ]
    sks = [
        0x0E5BD52621B6A8956086DCF0ECC89F0CDCA56CEBB2A8516C2D4252A9867FC551,
        0x19773A731561958A4F257B85AF81769BCB1146476936C4D9ADD796D4D3FDA020,
        0x6C9E69A6781538C945EAD231AECBEC9CF6CA3500DF59BC85F711FC97A768694E,
        0x2948F046357E74993187A6EF40ACB961911C52AC7A4257BABE6AF197F447E892,
    ]
    for i in range(4):
        assert bls.keygen_ietf(bytes([0xAA + i]) * 32) == sks[i]
        assert bls.g1_compress(bls.sk_to_pk(sks[i])).hex() == pks[i]
        assert bls.g1_compress(bls.g1_decompress(bytes.fromhex(pks[i]))).hex() == pks[i]


def test_mainnet_block_signatures_decompress():
    """Valid-point corpus: mainnet randao reveals / block signatures (reference
    packages/beacon-node/test/unit/sync/backfill/blocks.json, copied as tests/golden/mainnet_g2_points.json)
    and selection proofs (state-transition/test/unit/util/aggregator.test.ts:28,37)."""
    with open(os.path.join(GOLDEN, "mainnet_g2_points.json")) as fh:
        fx = json.load(fh)
    pts = fx["points"]
    assert len(pts) == len(set(pts)) >= 55 and fx["count_blocks_json"] == 53  # every G2 encoding blocks.json holds
    for h in pts:
        b = bytes.fromhex(h)
        pt = bls.signature_from_bytes(b)  # decompress + subgroup check, must not raise
        assert bls.g2_compress(pt) == b
        assert bls.g2_in_subgroup_def(pt)


def test_g2_infinity():
    """reference state-transition/test/unit/constants.test.ts:5-9."""
    inf = bytes([0xC0]) + bytes(95)
    assert bls.signature_from_bytes(inf) is None
    assert bls.g2_compress(None) == inf


def test_multithread_fixture_sets():
    """reference beacon-node/test/e2e/chain/bls/multithread.test.ts:28-41 and 89-106."""
    sets = []
    for i in range(3):
        sk = int.from_bytes(bytes([i + 1]) * 32, "big")
        msg = bytes([i + 1]) * 32
        sets.append((bls.sk_to_pk(sk), msg, bls.g2_compress(bls.sign(sk, msg))))
    assert bls.verify_signature_sets_maybe_batch(sets) is True
    assert bls.verify_signature_sets_maybe_batch(sets[:1]) is True
    with pytest.raises(bls.BlstError, match="BLST_INVALID_SIZE"):
        bls.verify_signature_sets_maybe_batch([(sets[0][0], sets[0][1], bytes(32))])
    with pytest.raises(ValueError, match="Empty signature set"):
        bls.verify_signature_sets_maybe_batch([])
    bad = [(sets[0][0], sets[1][1], sets[0][2])] + sets[1:]
    assert bls.verify_signature_sets_maybe_batch(bad) is False


def test_pairing_consistency():
    P1 = bls.g1_mul(bls.G1_GEN, 12345)
    Q1 = bls.g2_mul(bls.G2_GEN, 678)
    a = bls.final_exp(bls.f12conj(bls.miller_loop_affine(P1, Q1)))
    b = bls.final_exp(bls.miller_loop(P1, Q1))
    assert a == b
    c = bls.final_exp_def(bls.miller_loop(P1, Q1))
    assert bls.f12mul(bls.f12mul(c, c), c) == b
    e1 = bls.pairing(bls.G1_GEN, bls.G2_GEN)
    e2 = bls.pairing(bls.g1_mul(bls.G1_GEN, 6), bls.g2_mul(bls.G2_GEN, 7))
    assert e1 != bls.F12_ONE and bls.f12pow(e1, 42) == e2


def test_tower_against_polynomial_fp12():
    rnd = random.Random(3)
    rf2 = lambda: (rnd.randrange(bls.P), rnd.randrange(bls.P))
    x = ((rf2(), rf2(), rf2()), (rf2(), rf2(), rf2()))
    y = ((rf2(), rf2(), rf2()), (rf2(), rf2(), rf2()))
    assert bls.tower_to_poly(bls.f12mul(x, y)) == bls.poly_mul(bls.tower_to_poly(x), bls.tower_to_poly(y))
    assert bls.f12frob(x, 1) == bls.f12pow(x, bls.P)
    assert bls.f12mul(x, bls.f12inv(x)) == bls.F12_ONE


def test_isogeny_and_cofactor():
    rnd = random.Random(1)
    for _ in range(2):
        while True:
            xx = (rnd.randrange(bls.P), rnd.randrange(bls.P))
            y = bls.f2sqrt(bls.f2add(bls.f2mul(bls.f2add(bls.f2sqr(xx), bls.SSWU_A), xx), bls.SSWU_B))
            if y:
                break
        assert bls.on_curve(bls.Fp2Ops, bls.iso3_map((xx, y)))
        while True:
            xx = (rnd.randrange(bls.P), rnd.randrange(bls.P))
            y = bls.f2sqrt(bls.f2add(bls.f2mul(bls.f2sqr(xx), xx), bls.B2))
            if y:
                break
        pt = (xx, y)
        assert not bls.g2_in_subgroup_psi(pt) and not bls.g2_in_subgroup_def(pt)
        cc = bls.clear_cofactor_g2(pt)
        assert cc == bls.g2_mul(pt, bls.H_EFF_G2)
        assert bls.g2_in_subgroup_psi(cc)

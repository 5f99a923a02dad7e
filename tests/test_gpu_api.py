"""GPU tests of the callers on either side of the verifier path (lodestar_amd/api.py): the spec runner's
FastAggregateVerify entry points and KeyValidate on tests/golden/fav_cases.json (oracle-generated in the shape of
the consensus spec tests run by reference beacon-node/test/spec/general/bls.ts), verifySignatureSet
(signatureSets.ts:24-38) on the golden sets, and processDeposit's signature check (processDeposit.ts:54-64)
on the reference's interop deposit KAT."""
import json
import os

import pytest

from oracle import bls12_381 as bls
from oracle import ssz_min

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FAV = json.load(open(os.path.join(ROOT, "tests", "golden", "fav_cases.json")))
FX = json.load(open(os.path.join(ROOT, "tests", "golden", "verify_sets.json")))


@pytest.fixture(scope="module")
def ctx():
    from lodestar_amd.native import Context

    c = Context([0])
    yield c
    c.close()


@pytest.mark.parametrize("case", [c["name"] for c in FAV["cases"]])
def test_fast_aggregate_verify_cases(ctx, case):
    from lodestar_amd import api

    c = next(x for x in FAV["cases"] if x["name"] == case)
    pks = [bytes.fromhex(p) for p in c["pubkeys"]]
    msg, sig = bytes.fromhex(c["message"]), bytes.fromhex(c["signature"])
    assert api.fast_aggregate_verify(ctx, pks, msg, sig) is c["fast_aggregate_verify"]
    assert api.eth_fast_aggregate_verify(ctx, pks, msg, sig) is c["eth_fast_aggregate_verify"]
    if pks:
        _, st = api.key_validate(ctx, pks)
        assert list(st) == c["key_validate"]


def test_eth_aggregate_pubkeys(ctx):
    from lodestar_amd import api

    c = next(x for x in FAV["cases"] if x["name"] == "extra_key")
    pks = [bytes.fromhex(p) for p in c["pubkeys"]]
    want = bls.g1_compress(bls.aggregate_pubkeys([bls.g1_decompress(p) for p in pks]))
    assert api.eth_aggregate_pubkeys(ctx, pks) == want
    assert api.eth_aggregate_pubkeys(ctx, pks + [api.G1_INFINITY_48]) is None
    assert api.eth_aggregate_pubkeys(ctx, []) is None


def test_verify_signature_set_golden(ctx):
    """single -> Signature.verify, aggregate -> verifyAggregate; malformed signatures raise BLST errors."""
    from lodestar_amd import api

    keys = [bytes.fromhex(k["pk"]) for k in FX["keys"]]
    case = next(c for c in FX["cases"] if c["name"] == "each_alone/plain")
    for j, want in zip(case["jobs"], case["expected"]):
        s = FX["sets"][j[0]]
        pk = keys[s["pks"][0]] if len(s["pks"]) == 1 and not s["name"].startswith("aggregate") else [keys[i] for i in s["pks"]]
        args = (ctx, pk, bytes.fromhex(s["msg"]), bytes.fromhex(s["sig"]))
        if want < 0:
            with pytest.raises(api.BlstError) as e:
                api.verify_signature_set(*args)
            assert e.value.code == -want
        else:
            assert api.verify_signature_set(*args) is bool(want)


def test_process_deposit_signature_kat(ctx):
    """The interop deposit (genesisState.test.ts:51-55) is accepted; a corrupted signature, a wrong amount
    (other signing root), an invalid key and an infinity key are skipped (False, never raised)."""
    from lodestar_amd import api

    pk = bytes.fromhex("a99a76ed7796f7be22d5b7e85deeb7c5677e88e511e0b337618f8c4eb61349b4bf2d153f649f7b53359fe8b94a38e44c")
    sig = bytes.fromhex(
        "a95af8ff0f8c06af4d29aef05ce865f85f82df42b606008ec5b1bcb42b17ae47f4b78cdce1db31ce32d18f42a6b296b4"
        "014a2164981780e56b5a40d7723c27b8423173e58fa36f075078b177634f66351412b867c103f532aedd50bcd9b98446")
    wc = bytes.fromhex("00fad2a6bfb0e7f1f0f45460944fbd8dfa7f37da06a4d13b3983cc90bb46963b")
    domain = ssz_min.compute_domain(ssz_min.DOMAIN_DEPOSIT, bytes.fromhex("00000001"))
    root = ssz_min.compute_signing_root(ssz_min.deposit_message_root(pk, wc, 32_000_000_000), domain)
    other = ssz_min.compute_signing_root(ssz_min.deposit_message_root(pk, wc, 31_000_000_000), domain)
    bad_key = next(bytes.fromhex(p) for c in FAV["cases"] if c["name"] == "key_not_in_group" for p in c["pubkeys"][2:])
    assert api.process_deposit_signature(ctx, pk, root, sig) is True
    assert api.process_deposit_signature(ctx, pk, other, sig) is False
    assert api.process_deposit_signature(ctx, pk, root, bytes([0x00]) + sig[1:]) is False
    assert api.process_deposit_signature(ctx, bad_key, root, sig) is False
    assert api.process_deposit_signature(ctx, api.G1_INFINITY_48, root, sig) is False
    got = api.process_deposit_signatures(ctx, [pk, bad_key, pk, pk], [root, root, other, root],
                                         [sig, sig, sig, sig[:95]])
    assert got == [True, False, False, False]

"""GPU parity against the C restatement (oracle/blscpu.c, pinned by tests/test_cpu_oracle.py) at BASELINE.json's
own sizes, and the reference's known-answer data run through the kernels.

* C1 (128 single sets) and C2 at full size (16,384 single sets): every signature made by the ORACLE (not by
  the device), ~1% of sets corrupted in every way the reference distinguishes (wrong message, swapped
  signature, every Signature.fromBytes error class, the identity signature), then per-job results compared
  with the oracle's pool restatement on the identical batch, in table, bytes and bytes-aggregate modes.
* Reference KATs through the HIP path: the interop deposit (genesisState.test.ts:51-55: sign byte-equal,
  signing root, KeyValidate, verify), the mainnet G2 corpus (backfill/blocks.json: decode + subgroup +
  re-encode) and cachedKeys (cli/test/utils/cachedKeys.ts:15-26: KeyValidate, sk_to_pk, table upload).
* PublicKey.aggregate(...).toBytes() byte-identical to the golden fixture and the oracle (utils.ts:5-16).
* Message dedupe / same-message merging, KeyValidate classes, signing roots, two-shard sharding.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import bls12_381 as bls
from oracle import cpu, ssz_min

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FX = json.load(open(os.path.join(ROOT, "tests", "golden", "verify_sets.json")))
THREADS = min(16, os.cpu_count() or 1)  # the GPU box's CPU share
SEED = 0x4C4F444553544152

DEPOSIT_PK = bytes.fromhex("a99a76ed7796f7be22d5b7e85deeb7c5677e88e511e0b337618f8c4eb61349b4bf2d153f649f7b53359fe8b94a38e44c")
DEPOSIT_SIG = bytes.fromhex(
    "a95af8ff0f8c06af4d29aef05ce865f85f82df42b606008ec5b1bcb42b17ae47f4b78cdce1db31ce32d18f42a6b296b4"
    "014a2164981780e56b5a40d7723c27b8423173e58fa36f075078b177634f66351412b867c103f532aedd50bcd9b98446")
DEPOSIT_WC = bytes.fromhex("00fad2a6bfb0e7f1f0f45460944fbd8dfa7f37da06a4d13b3983cc90bb46963b")
DEPOSIT_ROOT = bytes.fromhex("f9e9adcff9c1517685beae7922ba8d8743626199d2bd7b397f3bd97ac140b542")
CACHED = [
    ("0e5bd52621b6a8956086dcf0ecc89f0cdca56cebb2a8516c2d4252a9867fc551",
     "8be678633e927aa0435addad5dcd5283fef6110d91362519cd6d43e61f6c017d724fa579cc4b2972134e050b6ba120c0"),
    ("19773a731561958a4f257b85af81769bcb1146476936c4d9add796d4d3fda020",
     "8e602f8ec17777c22f465f9b4707c2840647790f15f5c33bd8850f274d5c320850105639960ae4effe57aa5dd279bb98"),
    ("6c9e69a6781538c945ead231aecbec9cf6ca3500df59bc85f711fc97a768694e",
     "832a777fe5d89724583bcce5b4794d0b38be419a2daed09d7ee6af2c7c09465e0e2cd07a305c38e59e83e211e8ded246"),
    ("2948f046357e74993187a6ef40acb961911c52ac7a4257babe6af197f447e892",
     "8076b9d469d71902e06cce3af0528c190850d3dabfb8314eba1ef4eb789131de0dd75d2fe4b7964f347bfe61597cde54"),
]


@pytest.fixture(scope="module")
def ctx():
    from lodestar_amd.native import Context

    c = Context([0])
    yield c
    c.close()


def interop_sks(n, first=0):
    return b"".join(bls.interop_secret_key(i).to_bytes(32, "big") for i in range(first, first + n))


def msg(j, tag=b""):
    return hashlib.sha256(tag + SEED.to_bytes(8, "little") + j.to_bytes(4, "little")).digest()


def adversarial_sigs():
    """One signature per Signature.fromBytes error class (first candidates of a fixed scan) + infinity."""
    out = {}
    for t in range(1, 400):
        cand = bytes([0x80]) + bytes(45) + t.to_bytes(2, "big") + bytes(48)
        c = bls.classify_signature(cand)
        if c and c not in out:
            out[c] = cand
        if bls.BLST_POINT_NOT_ON_CURVE in out and bls.BLST_POINT_NOT_IN_GROUP in out:
            break
    out[bls.BLST_BAD_ENCODING] = bytes([0x80 | 0x1F]) + bytes([0xFF]) * 95  # x >= p
    return out


def corrupted_single_sets(n, tag, rng):
    """n oracle-signed single sets with ~1% corrupted: returns sks, pks (96 B), msgs, sigs (192-B stride),
    sig_len."""
    sks = interop_sks(n, first=int.from_bytes(hashlib.sha256(tag).digest()[:2], "little") % 1000)
    msgs = [msg(j, tag) for j in range(n)]
    sigs = cpu.sign(sks, b"".join(msgs), threads=THREADS)
    pks = cpu.sk_to_pk(sks, threads=THREADS)
    sig_list = [sigs[96 * i: 96 * i + 96] for i in range(n)]
    sig_len = [96] * n
    bad = rng.choice(n, size=max(8, n // 100), replace=False)
    adv = adversarial_sigs()
    kinds = ["wrong_msg", "swap", "infinity", "size"] + sorted(adv)
    for k, i in enumerate(bad.tolist()):
        kind = kinds[k % len(kinds)]
        if kind == "wrong_msg":
            msgs[i] = msg(i, tag + b"other")
        elif kind == "swap":
            j = (i + 1) % n
            sig_list[i] = sigs[96 * j: 96 * j + 96]
        elif kind == "infinity":
            sig_list[i] = bytes([0xC0]) + bytes(95)
        elif kind == "size":
            sig_list[i] = sig_list[i][:48]
            sig_len[i] = 48
        else:
            sig_list[i] = adv[kind]
    sig_buf = b"".join(s.ljust(192, b"\0") for s in sig_list)
    return sks, pks, msgs, sig_buf, sig_len


def compare(ctx, table=None, **batch):
    got, st = ctx.verify_raw(**batch)
    want, _ = cpu.verify_jobs(table=table, threads=THREADS, **batch)
    assert np.array_equal(got, want), f"{np.nonzero(got != want)[0][:10]} got {got[got != want][:10]} want {want[got != want][:10]}"
    return got, st


@pytest.mark.parametrize("n,tag", [(128, b"C1"), (16384, b"C2")])
def test_full_size_single_sets_vs_oracle(ctx, n, tag):
    """C1 (128 sets) and C2 (16,384 sets) at full size, oracle-signed, ~1% corrupted."""
    rng = np.random.default_rng(n)
    sks, pks, msgs, sigs, sig_len = corrupted_single_sets(n, tag, rng)
    base = dict(sigs=sigs, sig_len=sig_len, msgs=b"".join(msgs), sig_stride=192)
    # gossip shape: one batchable job per set, bytes mode
    got, st = compare(ctx, job_first_set=np.arange(n + 1), pk_bytes=pks, job_flags=np.ones(n), **base)
    assert (got == 1).sum() >= n - max(8, n // 100) and (got == 0).sum() >= 2 and (got < 0).sum() >= 4
    assert st.batch_retries >= 1
    # table mode (the bench's C2 shape)
    ctx.upload_pubkeys(0, pks)
    compare(ctx, table=cpu.Table(pks), job_first_set=np.arange(n + 1), set_pk_first=np.arange(n + 1),
            pk_index=np.arange(n), job_flags=np.ones(n), **base)
    # one verifySignatureSets call per 128 sets (the reference pool's job size), non-batchable
    jfs = np.arange(0, n + 1, 128)
    got, _ = compare(ctx, job_first_set=jfs, pk_bytes=pks, job_flags=np.zeros(len(jfs) - 1), **base)
    # a clean copy (all valid) verifies everywhere
    good = cpu.sign(sks, b"".join(msg(j, tag) for j in range(n)), threads=THREADS)
    res, st = ctx.verify_raw(np.arange(n + 1), good, [96] * n, b"".join(msg(j, tag) for j in range(n)),
                             pk_bytes=pks, job_flags=np.ones(n))
    assert (res == 1).all() and st.batch_retries == 0


def test_speculative_msm_large_idle_run_vs_oracle(ctx):
    """spec_large: a 16,384-set call on an idle device takes the speculative MSM (over the sets that decoded, on the
    other pair's message stream) -- the corrupted sets' groups must still come out job for job as the oracle's (their
    clean jobs re-checked with exact masks), and a clean call must pass without retries."""
    n, tag = 16384, b"SP"
    rng = np.random.default_rng(7)
    sks, pks, msgs, sigs, sig_len = corrupted_single_sets(n, tag, rng)
    base = dict(sigs=sigs, sig_len=sig_len, msgs=b"".join(msgs), sig_stride=192)
    old = ctx.get_option("spec_large")
    ctx.set_option("spec_large", 1)
    try:
        got, st = compare(ctx, job_first_set=np.arange(n + 1), pk_bytes=pks, job_flags=np.ones(n), **base)
        assert (got < 0).sum() >= 4 and st.batch_retries >= 1
        jfs = np.arange(0, n + 1, 128)
        compare(ctx, job_first_set=jfs, pk_bytes=pks, job_flags=np.ones(len(jfs) - 1), **base)
        good = cpu.sign(sks, b"".join(msg(j, tag) for j in range(n)), threads=THREADS)
        res, st = ctx.verify_raw(np.arange(n + 1), good, [96] * n, b"".join(msg(j, tag) for j in range(n)),
                                 pk_bytes=pks, job_flags=np.ones(n))
        assert (res == 1).all() and st.batch_retries == 0
    finally:
        ctx.set_option("spec_large", old)


def test_device_signing_matches_oracle(ctx):
    """The bench generates its workload with the device's sign / sk_to_pk ops: pin them to the oracle."""
    n = 256
    sks = interop_sks(n)
    msgs = b"".join(msg(j, b"sign") for j in range(n))
    dev_sigs, st = ctx.debug_op(7, b"".join(sks[32 * i: 32 * i + 32] + msgs[32 * i: 32 * i + 32] for i in range(n)),
                                64, 96)
    assert (st == 0).all() and dev_sigs == cpu.sign(sks, msgs, threads=THREADS)
    dev_pks, st = ctx.debug_op(8, sks, 32, 96)
    assert (st == 0).all() and dev_pks == cpu.sk_to_pk(sks, threads=THREADS)


def test_deposit_kat_through_kernels(ctx):
    """reference beacon-node/test/e2e/interop/genesisState.test.ts:51-55 on the GPU: signing root, KeyValidate
    of the 48-byte pubkey, sign byte-equal, verify true (and false on another root)."""
    from lodestar_amd.native import ROOT_OBJECT

    domain = ssz_min.compute_domain(ssz_min.DOMAIN_DEPOSIT, bytes.fromhex("00000001"))
    obj = ssz_min.deposit_message_root(DEPOSIT_PK, DEPOSIT_WC, 32_000_000_000)
    assert ctx.signing_roots(ROOT_OBJECT, obj, domain) == [DEPOSIT_ROOT]
    pk96, st = ctx.key_validate(DEPOSIT_PK, 48)
    assert st[0] == 0 and pk96 == cpu.sk_to_pk(bls.interop_secret_key(0).to_bytes(32, "big"))
    sig, st = ctx.debug_op(7, bls.interop_secret_key(0).to_bytes(32, "big") + DEPOSIT_ROOT, 64, 96)
    assert st[0] == 0 and sig == DEPOSIT_SIG
    res, _ = ctx.verify_raw([0, 1, 2], DEPOSIT_SIG * 2, [96, 96], DEPOSIT_ROOT + bytes(32), pk_bytes=pk96 * 2,
                            job_flags=[0, 0])
    assert list(res) == [1, 0]


def test_mainnet_g2_corpus_through_kernels(ctx):
    """Mainnet block signatures / randao reveals (reference backfill/blocks.json, aggregator.test.ts): the
    device decodes and subgroup-checks every one, and the decoded point re-encodes to the same bytes."""
    pts = [bytes.fromhex(h) for h in json.load(open(os.path.join(ROOT, "tests", "golden", "mainnet_g2_points.json")))["points"]]
    inp = b"".join(p.ljust(192, b"\0") + (96).to_bytes(2, "little") for p in pts)
    out, st = ctx.debug_op(1, inp, 194, 192)
    assert (st == 0).all()
    for i, p in enumerate(pts):
        x1, x0, y1, y0 = (int.from_bytes(out[192 * i + 48 * k: 192 * i + 48 * k + 48], "big") for k in range(4))
        assert bls.g2_compress(((x0, x1), (y0, y1))) == p


def test_cached_keys_through_kernels():
    """cli/test/utils/cachedKeys.ts:15-26: KeyValidate of the compressed keys, sk_to_pk byte-equal, and the
    decoded keys enter a fresh device table."""
    from lodestar_amd.native import Context

    c = Context([0])
    try:
        pk48 = b"".join(bytes.fromhex(p) for _, p in CACHED)
        pk96, st = c.key_validate(pk48, 48)
        assert (st == 0).all()
        dev, st = c.debug_op(8, b"".join(bytes.fromhex(s) for s, _ in CACHED), 32, 96)
        assert (st == 0).all() and dev == pk96
        for i in range(4):
            assert cpu.pk_decode(bytes.fromhex(CACHED[i][1])) == (0, pk96[96 * i: 96 * i + 96])
        c.upload_pubkeys(0, pk96)
        assert c.pubkeys_count == 4
        out, st = c.aggregate_pubkeys(set_pk_first=[0, 1, 2, 3, 4], pk_index=[0, 1, 2, 3], out_len=48)
        assert (st == 0).all() and [o.hex() for o in out] == [p for _, p in CACHED]
    finally:
        c.close()


def test_aggregate_pubkeys_golden_and_oracle(ctx):
    """PublicKey.aggregate(...).toBytes() byte-identical: golden fixture (table + bytes-aggregate modes, both
    encodings) and the oracle on random aggregates up to a 512-key committee, an empty set, a malformed key."""
    from lodestar_amd.native import Context

    keys = b"".join(bytes.fromhex(k["pk"]) for k in FX["keys"])
    spf, idx = [0], []
    for a in FX["aggregate_pubkeys"]:
        idx += a["pks"]
        spf.append(len(idx))
    c = Context([0])
    try:
        c.upload_pubkeys(0, keys)
        out, st = c.aggregate_pubkeys(set_pk_first=spf, pk_index=idx)
        assert (st == 0).all() and [o.hex() for o in out] == [a["pk"] for a in FX["aggregate_pubkeys"]]
        kb = b"".join(keys[96 * i: 96 * i + 96] for i in idx)
        out, st = c.aggregate_pubkeys(pk_bytes=kb, set_pk_first=spf)
        assert [o.hex() for o in out] == [a["pk"] for a in FX["aggregate_pubkeys"]]
        out48, _ = c.aggregate_pubkeys(pk_bytes=kb, set_pk_first=spf, out_len=48)
        assert out48 == [bls.g1_compress(bls.g1_deserialize(bytes.fromhex(a["pk"]))) for a in FX["aggregate_pubkeys"]]
    finally:
        c.close()
    rng = np.random.default_rng(5)
    pool = cpu.sk_to_pk(interop_sks(1024), threads=THREADS)
    sizes = [1, 2, 3, 64, 65, 127, 128, 511, 512, 0, 7]
    spf = np.concatenate([[0], np.cumsum(sizes)])
    sel = np.concatenate([rng.choice(1024, s, replace=False) for s in sizes]).astype(np.int64)
    kb = bytearray(b"".join(pool[96 * i: 96 * i + 96] for i in sel))
    kb[96 * (spf[-2] + 3)] |= 0x80  # set 10's fourth key: compressed flag on a 96-byte key -> BAD_ENCODING
    for out_len in (96, 48):
        got, gst = ctx.aggregate_pubkeys(pk_bytes=bytes(kb), set_pk_first=spf, out_len=out_len)
        want, wst = cpu.aggregate_pubkeys(out_len=out_len, job_first_set=[0, len(sizes)], sigs=bytes(96 * len(sizes)),
                                          sig_len=[96] * len(sizes), msgs=bytes(32 * len(sizes)), pk_bytes=bytes(kb),
                                          set_pk_first=spf)
        assert list(gst) == list(wst) and got == want
    assert gst[9] == 9 and gst[10] == bls.BLST_BAD_ENCODING  # EMPTY_AGGREGATE_ARRAY, malformed key


@pytest.mark.parametrize("n_sets", [2000, 5000, 9000])
def test_aggregate_pubkeys_lane_groups_vs_oracle(ctx, n_sets):
    """The aggregation's lane-group forms (k_pk_aggregate_g: 32 / 16 / 8 lanes per set, chosen by the number of sets,
    in-register butterfly) on many small aggregates in bytes-aggregate mode, with malformed keys at several positions
    and empty sets: statuses and both encodings byte-identical to the oracle."""
    rng = np.random.default_rng(n_sets)
    pool = cpu.sk_to_pk(interop_sks(512), threads=THREADS)
    sizes = rng.integers(0, 12, n_sets)
    spf = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    sel = rng.integers(0, 512, int(spf[-1]))
    kb = bytearray(b"".join(pool[96 * i: 96 * i + 96] for i in sel))
    for s in rng.choice(n_sets, 20, replace=False):
        if sizes[s] >= 2:
            kb[96 * (spf[s] + int(rng.integers(0, sizes[s])))] |= 0x80  # compressed flag on a 96-byte key
    for out_len in (96, 48):
        got, gst = ctx.aggregate_pubkeys(pk_bytes=bytes(kb), set_pk_first=spf, out_len=out_len)
        want, wst = cpu.aggregate_pubkeys(out_len=out_len, job_first_set=[0, n_sets], sigs=bytes(96 * n_sets),
                                          sig_len=[96] * n_sets, msgs=bytes(32 * n_sets), pk_bytes=bytes(kb),
                                          set_pk_first=spf, threads=THREADS)
        assert list(gst) == list(wst) and got == want
    assert (gst == bls.BLST_BAD_ENCODING).sum() >= 5 and (gst == 9).sum() >= 1


def test_bytes_aggregate_mode_golden(ctx):
    """Aggregate ISignatureSets from per-key bytes (any PublicKey objects, attestation.ts:131-138) on every
    golden case."""
    keys = [bytes.fromhex(k["pk"]) for k in FX["keys"]]
    for c in FX["cases"]:
        jfs, order = [0], []
        for j in c["jobs"]:
            order += j
            jfs.append(len(order))
        sets = [FX["sets"][k] for k in order]
        sigs = [bytes.fromhex(s["sig"]) for s in sets]
        spf, kb = [0], b""
        for s in sets:
            kb += b"".join(keys[i] for i in s["pks"])
            spf.append(spf[-1] + len(s["pks"]))
        res, _ = ctx.verify_raw(jfs, b"".join(x.ljust(192, b"\0")[:192] for x in sigs), [len(x) for x in sigs],
                                b"".join(bytes.fromhex(s["msg"]) for s in sets), pk_bytes=kb, set_pk_first=spf,
                                job_flags=[int(c["batchable"])] * len(c["jobs"]), sig_stride=192)
        assert list(res) == c["expected"], c["name"]


def test_dedupe_and_same_message_merging(ctx):
    """64 committees x 16 single-key sets sharing AttestationData roots, one wrong signature and one
    malformed one: identical per-job results with dedupe on and off, and vs the oracle; H(m) is computed
    once per root and the batch pass pairs once per (group, root)."""
    n_comm, per = 64, 16
    n = n_comm * per
    sks = interop_sks(n, first=3000)
    msgs = [msg(i // per, b"committee") for i in range(n)]
    sigs = bytearray(cpu.sign(sks, b"".join(msgs), threads=THREADS))
    pks = cpu.sk_to_pk(sks, threads=THREADS)
    sigs[96 * 100: 96 * 101] = sigs[96 * 101: 96 * 102]  # same committee, other signer
    sigs[96 * 700] = 0x00  # compressed flag cleared -> BAD_ENCODING
    batch = dict(job_first_set=np.arange(n + 1), sigs=bytes(sigs), sig_len=[96] * n, msgs=b"".join(msgs),
                 pk_bytes=pks, job_flags=np.ones(n))
    got, st = compare(ctx, **batch)
    assert got[100] == 0 and got[700] == -bls.BLST_BAD_ENCODING and (np.delete(got, [100, 700]) == 1).all()
    assert st.unique_messages == n_comm and st.pairing_units < n // 4
    ctx.set_option("dedupe", 0)
    try:
        got2, st2 = ctx.verify_raw(**batch)
    finally:
        ctx.set_option("dedupe", 1)
    assert np.array_equal(got, got2) and st2.unique_messages == n and st2.pairing_units == n


def test_key_validate_classes_vs_oracle(ctx):
    cands = [bytes([0xC0]) + bytes(47), bytes(48), bytes([0x9F]) + bytes([0xFF]) * 47]
    cands += [bytes([0x80 | (t & 0x20)]) + bytes(45) + t.to_bytes(2, "big") for t in range(1, 200)]
    cands += [bytes.fromhex(p) for _, p in CACHED]
    _, st = ctx.key_validate(b"".join(cands), 48)
    assert list(st) == [cpu.key_validate(c) for c in cands]
    assert len(set(st.tolist())) >= 5


def test_signing_roots_attestation_data(ctx):
    """computeSigningRoot(AttestationData, domain) (signingRoot.ts:7-13) vs the SSZ restatement."""
    from lodestar_amd.native import ROOT_ATTESTATION_DATA

    rng = np.random.default_rng(9)
    objs, want = [], []
    domain = ssz_min.compute_domain(bytes.fromhex("01000000"), bytes.fromhex("00000001"), bytes(range(32)))
    for _ in range(200):
        slot, index, se, te = (int(x) for x in rng.integers(0, 2**40, 4))
        bbr, sr, tr = (bytes(rng.integers(0, 256, 32, dtype=np.uint8)) for _ in range(3))
        objs.append(slot.to_bytes(8, "little") + index.to_bytes(8, "little") + bbr + se.to_bytes(8, "little") + sr
                    + te.to_bytes(8, "little") + tr)
        cp = lambda e, r: ssz_min.merkleize([ssz_min.uint64_root(e), r])
        root = ssz_min.merkleize([ssz_min.uint64_root(slot), ssz_min.uint64_root(index), bbr, cp(se, sr), cp(te, tr)])
        want.append(ssz_min.compute_signing_root(root, domain))
    assert ctx.signing_roots(ROOT_ATTESTATION_DATA, b"".join(objs), domain) == want


def test_two_shards_match_one():
    """The in-process multi-device path (jobs sharded over two device contexts, here both on device 0)
    gives the single-device answer job for job."""
    from lodestar_amd.native import Context

    n = 2048
    rng = np.random.default_rng(11)
    sks, pks, msgs, sigs, sig_len = corrupted_single_sets(n, b"shard", rng)
    batch = dict(job_first_set=np.arange(n + 1), sigs=sigs, sig_len=sig_len, msgs=b"".join(msgs), pk_bytes=pks,
                 job_flags=np.ones(n), sig_stride=192)
    c2 = Context([0, 0])
    try:
        c2.set_option("route_split_sets", 1024)  # 2,048 sets would otherwise run whole on one device
        got, st = c2.verify_raw(**batch)
        assert st.devices_used == 2
    finally:
        c2.close()
    want, _ = cpu.verify_jobs(threads=THREADS, **batch)
    assert np.array_equal(got, want)


def test_msm_exceptional_buckets_vs_oracle(ctx):
    """The bucket MSM (k_msm.hip) on inputs that hit its exceptional additions: one valid set repeated 600 times
    (every bucket adds the same point: doublings), sets whose signatures are each other's negation, groups of
    several MSM slices (> 256 sets), and a wrong signature among repeats (the fallback's per-job MSMs)."""
    sks = interop_sks(4, first=5000)
    pks = cpu.sk_to_pk(sks, threads=THREADS)
    m = [msg(j, b"msm") for j in range(4)]
    sig = cpu.sign(sks, b"".join(m), threads=THREADS)
    reps = 600
    idx = [0] * reps + [1, 2, 3]
    sigs = [sig[96 * i: 96 * i + 96] for i in idx]
    neg = bytes([sig[96] ^ 0x20]) + sig[97:192]  # the y-sign flag: -sig_1
    sigs += [neg]  # -sig_1 over m_1: false, and cancels sig_1 inside buckets
    idx += [1]
    sigs[300] = sig[96 * 2: 96 * 3]  # set 300 carries set 2's signature: false
    n = len(idx)
    batch = dict(job_first_set=np.arange(n + 1), sigs=b"".join(sigs), sig_len=[96] * n,
                 msgs=b"".join(m[i] for i in idx), pk_bytes=b"".join(pks[96 * i: 96 * i + 96] for i in idx),
                 job_flags=np.ones(n))
    got, st = compare(ctx, **batch)
    want = np.ones(n, np.int8)
    want[300] = 0
    want[n - 1] = 0
    assert np.array_equal(got, want) and st.batch_retries >= 1
    # all valid: one group of 603 sets (three MSM slices), no fallback
    ok = dict(batch, sigs=b"".join(sig[96 * i: 96 * i + 96] for i in idx[:-1]), sig_len=[96] * (n - 1),
              job_first_set=np.arange(n), msgs=b"".join(m[i] for i in idx[:-1]),
              pk_bytes=b"".join(pks[96 * i: 96 * i + 96] for i in idx[:-1]), job_flags=np.ones(n - 1))
    got, st = ctx.verify_raw(**ok)
    assert (got == 1).all() and st.batch_retries == 0


def test_merged_run_isolates_bad_call():
    """A call whose table index is beyond the device's table, queued between valid calls that a slot merges into one
    pipeline run, fails alone (ERR_ARGS) and never joins the run; the valid calls of the run keep their own answers
    (a bad call must not fail the calls merged with it)."""
    from concurrent.futures import ThreadPoolExecutor

    from lodestar_amd.native import Context

    n = 2048
    rng = np.random.default_rng(21)
    sks, pks, msgs, sigs, sig_len = corrupted_single_sets(n, b"merge", rng)
    c = Context([0])
    try:
        c.set_option("slots", 1)
        c.set_option("merge_sets", 1 << 20)
        c.upload_pubkeys(0, pks)
        assert c.get_option("slots") == 1
        good = dict(job_first_set=np.arange(n + 1), sigs=sigs, sig_len=sig_len, msgs=b"".join(msgs),
                    set_pk_first=np.arange(n + 1), pk_index=np.arange(n), job_flags=np.ones(n), sig_stride=192)
        bad_idx = np.arange(n)
        bad_idx[17] = n + 5  # beyond the 2048-entry table
        bad = dict(good, pk_index=bad_idx)
        want, _ = cpu.verify_jobs(table=cpu.Table(pks), threads=THREADS, **good)
        with ThreadPoolExecutor(8) as pool:
            futs = [pool.submit(c.verify_raw, **(bad if i in (2, 5) else good)) for i in range(8)]
            outs = []
            for i, f in enumerate(futs):
                try:
                    outs.append(f.result())
                except RuntimeError as e:
                    outs.append(e)
        for i, o in enumerate(outs):
            if i in (2, 5):
                assert isinstance(o, RuntimeError) and "ERR_ARGS" in str(o)
            else:
                assert np.array_equal(o[0], want), i
        assert max(o[1].run_calls for i, o in enumerate(outs) if i not in (2, 5)) >= 2  # some calls were merged
        # slots resize both ways and report the count in use
        c.set_option("slots", 3)
        assert c.get_option("slots") == 3
        c.set_option("slots", 2)
        assert c.get_option("slots") == 2
        got, _ = c.verify_raw(**good)
        assert np.array_equal(got, want)
    finally:
        c.close()


@pytest.mark.parametrize("k,lanes", [(2, 2), (4, 2), (2, 1), (1, 1), (1, 6), (2, 6), (3, 6), (1, 3), (2, 3), (3, 3)])
def test_miller_chunk_forms_vs_oracle(ctx, k, lanes):
    """The Miller accumulation's chunk forms: chunks of k pairings on six lanes (one w-basis coefficient of f each),
    two lanes (halves of f, the squaring shared by the chunk), lane pairs (lanes 3: every Fp2 split, gtx.hpp) or one
    lane, forced on a 2,048-set call with ~1% corrupted
    sets (so the fallback re-checks jobs through the same kernels): job for job equal to the oracle.  (coop_max 0: the
    lane forms even for a run this small.)"""
    n = 2048
    rng = np.random.default_rng(n + 17 * k + lanes)
    sks, pks, msgs, sigs, sig_len = corrupted_single_sets(n, b"MK", rng)
    base = dict(sigs=sigs, sig_len=sig_len, msgs=b"".join(msgs), sig_stride=192)
    coop = ctx.get_option("coop_max")
    ctx.set_option("miller_k", k)
    ctx.set_option("miller_lanes", lanes)
    ctx.set_option("coop_max", 0)
    try:
        got, st = compare(ctx, job_first_set=np.arange(n + 1), pk_bytes=pks, job_flags=np.ones(n), **base)
    finally:
        ctx.set_option("miller_k", 0)
        ctx.set_option("miller_lanes", 0)
        ctx.set_option("coop_max", coop)
    assert (got == 1).sum() >= n - max(8, n // 100) and st.batch_retries >= 1


@pytest.mark.parametrize("slice_len,tree", [(8, 1), (32, 1), (32, 0), (128, 1)])
def test_msm_slice_forms_vs_oracle(ctx, slice_len, tree):
    """The MSM of 1k-32k-set runs at other slice lengths, with and without the pairwise slice tree, on a 2,048-set
    call with ~1% corrupted sets: job for job equal to the oracle."""
    n = 2048
    rng = np.random.default_rng(7 * slice_len + tree)
    sks, pks, msgs, sigs, sig_len = corrupted_single_sets(n, b"MS", rng)
    base = dict(sigs=sigs, sig_len=sig_len, msgs=b"".join(msgs), sig_stride=192)
    ctx.set_option("msm_slice_mid", slice_len)
    ctx.set_option("msm_tree", tree)
    try:
        got, st = compare(ctx, job_first_set=np.arange(n + 1), pk_bytes=pks, job_flags=np.ones(n), **base)
    finally:
        ctx.set_option("msm_slice_mid", 32)
        ctx.set_option("msm_tree", 1)
    assert (got == 1).sum() >= n - max(8, n // 100) and st.batch_retries >= 1


def test_balanced_merging_keeps_answers():
    """merge_balance cuts a backlog of queued calls into equal runs; every call keeps its own answer."""
    from concurrent.futures import ThreadPoolExecutor

    from lodestar_amd.native import Context

    n = 1024
    rng = np.random.default_rng(33)
    sks, pks, msgs, sigs, sig_len = corrupted_single_sets(n, b"bal", rng)
    c = Context([0])
    try:
        c.set_option("merge_balance", 1)
        c.set_option("merge_sets", 3 * n)
        c.upload_pubkeys(0, pks)
        call = dict(job_first_set=np.arange(n + 1), sigs=sigs, sig_len=sig_len, msgs=b"".join(msgs),
                    set_pk_first=np.arange(n + 1), pk_index=np.arange(n), job_flags=np.ones(n), sig_stride=192)
        want, _ = cpu.verify_jobs(table=cpu.Table(pks), threads=THREADS, **call)
        with ThreadPoolExecutor(10) as pool:
            outs = [f.result() for f in [pool.submit(c.verify_raw, **call) for _ in range(10)]]
        for got, st in outs:
            assert np.array_equal(got, want)
    finally:
        c.close()


@pytest.mark.parametrize("lanes", [1, 2])
def test_two_lane_lines_vs_oracle(ctx, lanes):
    """The Miller lines on one lane per message (k_miller_lines) and on lane pairs (k_miller_lines2, fp2x.hpp; the
    default lines_lanes 2) on a 2,048-set call with ~1% corrupted sets: job for job equal to the oracle."""
    n = 2048
    rng = np.random.default_rng(99)
    sks, pks, msgs, sigs, sig_len = corrupted_single_sets(n, b"L2", rng)
    base = dict(sigs=sigs, sig_len=sig_len, msgs=b"".join(msgs), sig_stride=192)
    saved = ctx.get_option("lines_lanes")
    ctx.set_option("lines_lanes", lanes)
    try:
        got, st = compare(ctx, job_first_set=np.arange(n + 1), pk_bytes=pks, job_flags=np.ones(n), **base)
    finally:
        ctx.set_option("lines_lanes", saved)
    assert (got == 1).sum() >= n - max(8, n // 100)

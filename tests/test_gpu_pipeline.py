"""GPU parity tests: every stage of the HIP pipeline and the C-ABI verify path against the oracle.
Run on the MI355X box:  python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread"""
import hashlib
import random

import numpy as np
import pytest

from oracle import bls12_381 as bls
from tests.emu_helpers import b2f12, b2g1, b2g2, f12b, fpb, fromb, g1b, g2b, r_of_word

pytestmark = pytest.mark.gpu

P = bls.P
SEED = 0x4C4F444553544152


@pytest.fixture(scope="module")
def ctx():
    from lodestar_amd.native import Context

    c = Context()
    # these tests count groups and retries of a fixed grouping (multithread.test.ts:89-106 shapes): no adaptive sizing
    c.set_option("group_adapt", 0)
    yield c
    c.close()


def msg_j(j, seed=SEED):
    return hashlib.sha256(seed.to_bytes(8, "little") + j.to_bytes(4, "little")).digest()


def test_debug_fp_mul(ctx):
    rnd = random.Random(7)
    pairs = [(rnd.randrange(P), rnd.randrange(P)) for _ in range(200)] + [(P - 1, P - 1), (0, 5), (1, P - 1)]
    inp = b"".join(fpb(a) + fpb(b) for a, b in pairs)
    out, st = ctx.debug_op(0, inp, 96, 48)
    for k, (a, b) in enumerate(pairs):
        assert fromb(out[48 * k : 48 * k + 48]) == a * b % P


def test_debug_sig_decode(ctx):
    sig = bls.sign(0x1234567, b"\x07" * 32)
    cases = [bls.g2_compress(sig), bls.g2_serialize(sig), bytes(32), bytes([0xC0]) + bytes(95),
             bytes([0xE0]) + bytes(95), bytes([0x9A]) + b"\xff" * 95]
    for t in range(1, 30):
        cases.append(bytes([0x80]) + bytes(46) + bytes([t]) + bytes(48))
    inp = b""
    for c in cases:
        rec = c.ljust(192, b"\x00") + len(c).to_bytes(2, "little")
        inp += rec
    out, st = ctx.debug_op(1, inp, 194, 192)
    for k, c in enumerate(cases):
        want = bls.classify_signature(c)
        got = int(st[k])
        if got == -1:  # infinity
            assert bls.signature_from_bytes(c) is None
            continue
        assert got == want, (k, c.hex()[:20], got, want)
        if want == 0:
            assert b2g2(out[192 * k : 192 * k + 192]) == bls.signature_from_bytes(c)


def test_debug_hash_to_g2(ctx):
    msgs = [msg_j(j) for j in range(64)] + [bytes(32), b"\xff" * 32]
    out, st = ctx.debug_op(2, b"".join(msgs), 32, 192)
    for k, m in enumerate(msgs[:12] + msgs[-2:]):
        idx = msgs.index(m)
        assert st[idx] == 0
        assert b2g2(out[192 * idx : 192 * idx + 192]) == bls.hash_to_g2(m)


def test_debug_miller_final_exp(ctx):
    rnd = random.Random(3)
    pts = [(bls.g1_mul(bls.G1_GEN, rnd.randrange(1, bls.R)), bls.g2_mul(bls.G2_GEN, rnd.randrange(1, bls.R)))
           for _ in range(3)]
    inp = b"".join(g1b(p) + g2b(q) for p, q in pts)
    out, st = ctx.debug_op(3, inp, 288, 576)
    fs = []
    for k, (p, q) in enumerate(pts):
        f = b2f12(out[576 * k : 576 * k + 576])
        assert f == bls.miller_loop(p, q)
        fs.append(f)
    out2, _ = ctx.debug_op(4, b"".join(f12b(f) for f in fs), 576, 576)
    for k, f in enumerate(fs):
        assert b2f12(out2[576 * k : 576 * k + 576]) == bls.final_exp(f)


def test_debug_gt_wave(ctx):
    """Workgroup-cooperative Miller loop / final exponentiation (gt_wave.hpp, used by k_group_check) against
    the oracle, including a Miller loop with an addition-heavy path (the 5 addition steps of |z|)."""
    rnd = random.Random(5)
    pts = [(bls.g1_mul(bls.G1_GEN, rnd.randrange(1, bls.R)), bls.g2_mul(bls.G2_GEN, rnd.randrange(1, bls.R)))
           for _ in range(3)]
    pts.append((bls.g1_neg(bls.G1_GEN), pts[0][1]))
    out, st = ctx.debug_op(17, b"".join(g1b(p) + g2b(q) for p, q in pts), 288, 576)
    assert (st == 0).all()
    fs = []
    for k, (p, q) in enumerate(pts):
        f = b2f12(out[576 * k : 576 * k + 576])
        assert f == bls.miller_loop(p, q), k
        fs.append(f)
    fs.append(bls.f12mul(fs[0], fs[1]))
    out2, st2 = ctx.debug_op(16, b"".join(f12b(f) for f in fs), 576, 576)
    assert (st2 == 0).all()
    for k, f in enumerate(fs):
        assert b2f12(out2[576 * k : 576 * k + 576]) == bls.final_exp(f), k


def test_debug_scalar_mul(ctx):
    rnd = random.Random(11)
    Pp = bls.g1_mul(bls.G1_GEN, 99)
    Q = bls.g2_mul(bls.G2_GEN, 77)
    ks = [1, 2, 3, 0xFFFFFFFFFFFFFFFF] + [rnd.getrandbits(64) for _ in range(12)]
    out, st = ctx.debug_op(5, b"".join(g1b(Pp) + k.to_bytes(8, "little") for k in ks), 104, 96)
    for i, k in enumerate(ks):
        assert b2g1(out[96 * i : 96 * i + 96]) == bls.g1_mul(Pp, k)
    out, st = ctx.debug_op(6, b"".join(g2b(Q) + k.to_bytes(8, "little") for k in ks[:6]), 200, 192)
    for i, k in enumerate(ks[:6]):
        assert b2g2(out[192 * i : 192 * i + 192]) == bls.g2_mul(Q, k)


# ---------------------------------------------------------------------------- verify (C-ABI)
def make_sets(n, seed=SEED, start=0):
    out = []
    for j in range(start, start + n):
        sk = bls.interop_secret_key(j)
        m = msg_j(j, seed)
        pk = bls.sk_to_pk(sk)
        out.append((sk, pk, m, bls.g2_compress(bls.sign(sk, m))))
    return out


@pytest.fixture(scope="module")
def sets16():
    return make_sets(16)


def run_bytes_mode(ctx, sets, jobs, batchable=None, sigs_override=None, **kw):
    jfs = [0]
    for j in jobs:
        jfs.append(jfs[-1] + j)
    assert jfs[-1] == len(sets)
    sig_list = sigs_override or [s[3] for s in sets]
    stride = 192
    sigs = b"".join(s.ljust(stride, b"\x00")[:stride] for s in sig_list)
    sig_len = [len(s) for s in sig_list]
    msgs = b"".join(s[2] for s in sets)
    pkb = b"".join(bls.g1_serialize(s[1]) for s in sets)
    flags = None if batchable is None else [1 if b else 0 for b in batchable]
    return ctx.verify_raw(jfs, sigs, sig_len, msgs, pk_bytes=pkb, job_flags=flags, sig_stride=stride, **kw)


def test_verify_single_and_batch(ctx, sets16):
    res, st = run_bytes_mode(ctx, sets16, [1] * 16)
    assert list(res) == [1] * 16
    res, st = run_bytes_mode(ctx, sets16, [16])
    assert list(res) == [1]
    res, st = run_bytes_mode(ctx, sets16, [1] * 16, batchable=[True] * 16)
    assert list(res) == [1] * 16
    assert st.groups == 1 and st.batch_retries == 0


def test_verify_invalid_isolation(ctx, sets16):
    """multithread.test.ts:89-106: an invalid job does not make the others fail."""
    sigs = [s[3] for s in sets16]
    sigs[0] = bytes(32)  # BLST_INVALID_SIZE
    sigs[5] = sets16[6][3]  # well-formed, wrong signature -> false
    res, st = run_bytes_mode(ctx, sets16, [1] * 16, batchable=[True] * 16, sigs_override=sigs)
    want = [-8] + [1] * 4 + [0] + [1] * 10
    assert list(res) == want
    assert st.batch_retries == 1
    # non-batchable multi-set job containing the wrong signature -> false, others true
    res, st = run_bytes_mode(ctx, sets16, [4, 4, 8], sigs_override=[s[3] for s in sets16[:5]] + [sets16[6][3]] + [s[3] for s in sets16[6:]])
    assert list(res) == [1, 0, 1]


def test_verify_error_classes(ctx, sets16):
    sigs = [s[3] for s in sets16]
    sigs[1] = bytes([0xC0]) + bytes(95)  # infinity -> false
    sigs[2] = bytes([0xE0]) + bytes(95)  # bad encoding
    x = None
    for t in range(1, 60):
        cand = bytes([0x80]) + bytes(46) + bytes([t]) + bytes(48)
        c = bls.classify_signature(cand)
        if c == bls.BLST_POINT_NOT_ON_CURVE and x is None:
            x = cand
        if c == bls.BLST_POINT_NOT_IN_GROUP:
            sigs[4] = cand
    sigs[3] = x
    sigs[6] = bls.g2_serialize(bls.signature_from_bytes(sets16[6][3]))  # 192-byte form, valid
    res, _ = run_bytes_mode(ctx, sets16, [1] * 16, batchable=[True] * 16, sigs_override=sigs)
    assert list(res[:7]) == [1, 0, -1, -2, -3, 1, 1]
    assert all(r == 1 for r in res[7:])


def test_verify_empty_job(ctx, sets16):
    res, _ = run_bytes_mode(ctx, sets16[:2], [0, 2, 0])
    assert list(res) == [-10, 1, -10]


def test_verify_table_mode_aggregate(ctx):
    n_keys = 40
    sks = [bls.interop_secret_key(i) for i in range(n_keys)]
    pks = [bls.sk_to_pk(s) for s in sks]
    ctx.upload_pubkeys(0, b"".join(bls.g1_serialize(p) for p in pks))
    assert ctx.pubkeys_count >= n_keys
    # aggregate sets: same message signed by several keys; aggregate signature = (sum sk) H(m)
    groups = [list(range(0, 7)), list(range(7, 8)), list(range(8, 40)), [3, 3, 5]]
    sets = []
    for gi, g in enumerate(groups):
        m = msg_j(1000 + gi)
        sk_sum = sum(sks[i] for i in g) % bls.R
        sig = bls.g2_compress(bls.sign(sk_sum, m))
        sets.append((g, m, sig))
    jfs = list(range(len(sets) + 1))
    set_pk_first = [0]
    pk_index = []
    for g, _, _ in sets:
        pk_index += g
        set_pk_first.append(len(pk_index))
    sigs = b"".join(s[2] for s in sets)
    msgs = b"".join(s[1] for s in sets)
    res, _ = ctx.verify_raw(jfs, sigs, [96] * len(sets), msgs, set_pk_first=set_pk_first, pk_index=pk_index,
                            sig_stride=96)
    assert list(res) == [1, 1, 1, 1]
    # empty aggregate -> EMPTY_AGGREGATE_ARRAY
    res, _ = ctx.verify_raw([0, 1, 2], sigs[:192], [96, 96], msgs[:64], set_pk_first=[0, 7, 7],
                            pk_index=list(range(7)), sig_stride=96)
    assert list(res) == [1, -9]


def test_debug_scalar_word_mul():
    """The batch scalar of word w is r = a + b lambda (k_common.hpp jac_mul_scalar_word, tests/emu_helpers.py
    r_of_word): G1 and G2 against the oracle's plain scalar multiplication, including the extreme words."""
    from lodestar_amd.native import Context

    ctx = Context([0])
    try:
        rnd = random.Random(21)
        words = [0, 1, 2**64 - 1, 2**63, 0x0F0F0F0F0F0F0F0F] + [rnd.getrandbits(64) for _ in range(11)]
        P = bls.g1_mul(bls.G1_GEN, 987654321)
        Q = bls.g2_mul(bls.G2_GEN, 123456789)
        inp1 = b"".join(bls.g1_serialize(P) + w.to_bytes(8, "little") for w in words)
        inp2 = b"".join(bls.g2_serialize(Q) + w.to_bytes(8, "little") for w in words)
        o1, s1 = ctx.debug_op(10, inp1, 104, 1440)
        o2, s2 = ctx.debug_op(9, inp2, 200, 2880)
        assert (s1 == 0).all() and (s2 == 0).all()
        for k, w in enumerate(words):
            r = r_of_word(w, raw=True)  # the op scales by the digits of every word, 0 included
            assert o1[1440 * k: 1440 * k + 96] == bls.g1_serialize(bls.g1_mul(P, r))
            assert o2[2880 * k: 2880 * k + 192] == bls.g2_serialize(bls.g2_mul(Q, r))
    finally:
        ctx.close()


def test_fp_lc_device_edges(ctx):
    """fp_lc (fp.hpp) on the device (its MAD chain is inline assembly, so the host build does not cover it): terms at the
    edges of the contract (0, 1, p - 1, p, 2p - 1, 2p, random <= 2p) -- the combination mod p, normalized, < 1.003 p."""
    import random

    from oracle import bls12_381 as bls

    P = bls.P
    rnd = random.Random(12)
    edges = [0, 1, P - 1, P, 2 * P - 1, 2 * P]
    cases = [[2 * P if (k < 7) == (t % 2 == 0) else 0 for k in range(15)] for t in range(2)]
    cases += [[rnd.choice(edges) if rnd.random() < 0.5 else rnd.randrange(0, 2 * P + 1) for _ in range(15)]
              for _ in range(4094)]
    limbs = lambda v: [(v >> (28 * i)) & ((1 << 28) - 1) for i in range(13)] + [v >> (28 * 13)]
    inp = b"".join(np.array(sum((limbs(x) for x in xs), []), np.uint32).tobytes() for xs in cases)
    out, st = ctx.debug_op(11, inp, 15 * 56, 56)
    assert (st == 0).all()
    res = np.frombuffer(out, np.uint32).reshape(-1, 14)
    for xs, r in zip(cases, res):
        v = sum(int(x) << (28 * i) for i, x in enumerate(r))
        assert (r[:13] < (1 << 28)).all() and v < 1.003 * P
        assert v % P == (sum(xs[:7]) - sum(xs[7:])) % P


def test_lane_pair_g2_arithmetic_vs_one_lane(ctx):
    """The lane-pair G2 formulas (fp2x.hpp: hash_clear2, sig_subgroup2, msm_bucket2, miller_lines2) against the one-lane
    forms on the same points, including the addition's exceptional branches (P + P, P + (-P), infinity operands) and
    Jacobian inputs with Z != 1 (debug op 18), over the reference-held mainnet G2 corpus; [|z|]P also against the
    oracle."""
    import json
    import os

    pts = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "mainnet_g2_points.json")))["points"]
    aff = [bls.signature_from_bytes(bytes.fromhex(h), validate=False) for h in pts]
    n = len(aff)
    inp = b"".join(g2b(aff[i]) + g2b(aff[(i + 1) % n]) for i in range(n))
    out, st = ctx.debug_op(18, inp, 384, 192)
    assert (st == 0).all(), st
    for i in range(n):  # [|z|]P by the oracle
        want = bls.g2_mul(aff[i], bls.BLS_X_ABS)
        assert out[192 * i: 192 * i + 192] == g2b(want)
    with pytest.raises(RuntimeError, match="ERR_ARGS"):
        ctx.debug_op(18, inp, 383, 192)  # a stride below the op's element is refused on the host

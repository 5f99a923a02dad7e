"""The device arithmetic (lodestar_amd/csrc/*.hpp), compiled for the host CPU by tests/native/emu.cpp,
checked against the oracle.  Same source as the HIP kernels; the GPU parity tests re-check it on MI355X."""
import ctypes
import random

import pytest

from oracle import bls12_381 as bls
from tests.emu_helpers import (b2f12, b2f2, b2g1, b2g2, f12b, f2b, fpb, fromb, g1b, g2b, lib)

P = bls.P
rnd = random.Random(1234)


def buf(n):
    return ctypes.create_string_buffer(n)


def edge_fp():
    return [0, 1, 2, P - 1, P - 2, (P - 1) // 2, (P + 1) // 2, 2**380, 2**381 - 1 - P if 2**381 > P else 5,
            0xFFFFFFF, 1 << 28, (1 << 364) - 1] + [rnd.randrange(P) for _ in range(40)]


def test_fp_ops():
    L = lib()
    vals = edge_fp()
    o = buf(48)
    for a in vals:
        for b in vals[:12] + [rnd.randrange(P) for _ in range(3)]:
            L.emu_fp_mul(fpb(a), fpb(b), o)
            assert fromb(o.raw) == a * b % P, (a, b)
            L.emu_fp_add(fpb(a), fpb(b), o)
            assert fromb(o.raw) == (a + b) % P
            L.emu_fp_sub(fpb(a), fpb(b), o)
            assert fromb(o.raw) == (a - b) % P
        L.emu_fp_sqr(fpb(a), o)
        assert fromb(o.raw) == a * a % P
        L.emu_fp_half(fpb(a), o)
        assert fromb(o.raw) * 2 % P == a % P
    for a in vals[:10]:
        L.emu_fp_inv(fpb(a), o)
        assert fromb(o.raw) == (pow(a, P - 2, P))


def test_fp_inv_divsteps_edges_and_random():
    """fp_inv (Bernstein-Yang divsteps, fp.hpp) against x^(p-2) at the edges of its 40-batch bound: 0, 1, 2, p - 1,
    powers of two, values whose gcd chain is long (Fibonacci-like neighbours of p), all-ones limbs, and 1,500 random
    elements."""
    L = lib()
    o = buf(48)
    fib = [1, 1]
    while fib[-1] < P:
        fib.append(fib[-1] + fib[-2])
    vals = [0, 1, 2, 3, P - 1, P - 2, (P - 1) // 2, (P + 1) // 2, 2**380 % P, 2**28, 2**364 % P, (2**381 - 1) % P,
            int("0fffffff" * 12, 16) % P, fib[-2] % P, fib[-3] % P, (P * fib[-4]) // fib[-3]]
    vals += [2**k % P for k in range(0, 381, 17)]
    r2 = random.Random(2024)
    vals += [r2.randrange(P) for _ in range(1500)]
    for a in vals:
        L.emu_fp_inv(fpb(a), o)
        assert fromb(o.raw) == (pow(a, P - 2, P) if a % P else 0), a


def test_fp2_ops_and_sqrt():
    L = lib()
    o = buf(96)
    cases = [(0, 0), (1, 0), (0, 1), (P - 1, 0), (0, P - 1), (4, 0), (5, 0)] + [
        (rnd.randrange(P), rnd.randrange(P)) for _ in range(30)
    ] + [(rnd.randrange(P), 0) for _ in range(6)] + [(0, rnd.randrange(P)) for _ in range(6)]
    for a in cases:
        b = (rnd.randrange(P), rnd.randrange(P))
        L.emu_fp2_mul(f2b(a), f2b(b), o)
        assert b2f2(o.raw) == bls.f2mul(a, b)
        L.emu_fp2_sqr(f2b(a), o)
        assert b2f2(o.raw) == bls.f2sqr(a)
        if a != (0, 0):
            L.emu_fp2_inv(f2b(a), o)
            assert bls.f2mul(b2f2(o.raw), a) == (1, 0)
        ok = L.emu_fp2_sqrt(f2b(a), o)
        assert bool(ok) == bls.f2_is_square(a), a
        if ok:
            assert bls.f2sqr(b2f2(o.raw)) == a


def test_fp12_ops():
    L = lib()
    rf2 = lambda: (rnd.randrange(P), rnd.randrange(P))
    rf12 = lambda: ((rf2(), rf2(), rf2()), (rf2(), rf2(), rf2()))
    o = buf(576)
    for _ in range(3):
        a, b = rf12(), rf12()
        L.emu_fp12_mul(f12b(a), f12b(b), o)
        assert b2f12(o.raw) == bls.f12mul(a, b)
        L.emu_fp12_sqr(f12b(a), o)
        assert b2f12(o.raw) == bls.f12sqr(a)
        L.emu_fp12_inv(f12b(a), o)
        assert b2f12(o.raw) == bls.f12inv(a)
        L.emu_fp12_frob1(f12b(a), o)
        assert b2f12(o.raw) == bls.f12frob(a, 1)
        # cyclotomic squaring agrees with plain squaring on the cyclotomic subgroup (after the easy part)
        c = bls.f12mul(bls.f12conj(a), bls.f12inv(a))
        c = bls.f12mul(bls.f12frob(c, 2), c)
        L.emu_fp12_cyc_sqr(f12b(c), o)
        assert b2f12(o.raw) == bls.f12sqr(c)


def test_expand_and_hash_to_field():
    import os
    L = lib()
    o = buf(256)
    for i in range(5):
        msg = os.urandom(32) if i else bytes(32)
        L.emu_expand_message(msg, o)
        assert o.raw == bls.expand_message_xmd(msg, bls.DST_POP, 256)
        o2 = buf(192)
        L.emu_hash_to_field(msg, o2)
        u0, u1 = bls.hash_to_field_fp2(msg, 2)
        assert b2f2(o2.raw[:96]) == u0 and b2f2(o2.raw[96:]) == u1


def test_hash_to_g2():
    L = lib()
    o = buf(192)
    for i in range(4):
        msg = bytes([i]) * 32
        assert L.emu_hash_to_g2(msg, o) == 1
        assert b2g2(o.raw) == bls.hash_to_g2(msg)


def test_subgroup_and_scalar_mul():
    L = lib()
    o = buf(192)
    Q = bls.g2_mul(bls.G2_GEN, 987654321)
    assert L.emu_g2_in_subgroup(g2b(Q)) == 1
    assert L.emu_g2_in_subgroup_ld(g2b(Q)) == 1
    # random non-subgroup point
    while True:
        x = (rnd.randrange(P), rnd.randrange(P))
        y = bls.f2sqrt(bls.f2add(bls.f2mul(bls.f2sqr(x), x), bls.B2))
        if y:
            break
    assert L.emu_g2_in_subgroup(g2b((x, y))) == 0
    assert L.emu_g2_in_subgroup_ld(g2b((x, y))) == 0
    for k in [1, 2, 3, 0xFFFFFFFFFFFFFFFF, rnd.getrandbits(64)]:
        assert L.emu_g2_mul_u64(g2b(Q), k, o) == 1
        assert b2g2(o.raw) == bls.g2_mul(Q, k)
        o1 = buf(96)
        Pp = bls.g1_mul(bls.G1_GEN, 5555)
        assert L.emu_g1_mul_u64(g1b(Pp), k, o1) == 1
        assert b2g1(o1.raw) == bls.g1_mul(Pp, k)


def test_miller_and_final_exp():
    L = lib()
    Pp = bls.g1_mul(bls.G1_GEN, 12345)
    Q = bls.g2_mul(bls.G2_GEN, 678)
    o = buf(576)
    L.emu_miller(g1b(Pp), g2b(Q), o)
    f = b2f12(o.raw)
    assert f == bls.miller_loop(Pp, Q)
    o3 = buf(576)
    L.emu_miller2(g1b(Pp), g2b(Q), o3)  # two-pass pipeline form: lines of H(m), then the Fp12 fold
    assert b2f12(o3.raw) == f
    o2 = buf(576)
    L.emu_final_exp(f12b(f), o2)
    assert b2f12(o2.raw) == bls.final_exp(f)
    o4 = buf(576)  # the cooperative loop's phase schedule (gt_wave.hpp: f and the next line on separate waves)
    L.emu_gtw_miller(g1b(Pp), g2b(Q), o4)
    assert b2f12(o4.raw) == f


def test_sig_decode_classes():
    L = lib()
    o = buf(192)
    inf = ctypes.c_int()
    sk = 0x1234567
    sig = bls.sign(sk, b"\x07" * 32)
    comp = bls.g2_compress(sig)
    unc = bls.g2_serialize(sig)
    assert L.emu_sig_decode(comp, 96, o, ctypes.byref(inf)) == 0 and b2g2(o.raw) == sig
    assert L.emu_sig_decode(unc, 192, o, ctypes.byref(inf)) == 0 and b2g2(o.raw) == sig
    cases = {
        bytes(32): bls.BLST_INVALID_SIZE,
        bytes([0xC0]) + bytes(95): 0,
        bytes([0xE0]) + bytes(95): bls.BLST_BAD_ENCODING,
        bytes([0xC0]) + bytes(94) + b"\x01": bls.BLST_BAD_ENCODING,
        comp[:1].replace(comp[:1], bytes([comp[0] & 0x7F])) + comp[1:]: bls.BLST_BAD_ENCODING,
        bytes([0x9A]) + b"\xff" * 95: bls.BLST_BAD_ENCODING,  # x1 >= p
    }
    # non-residue x
    for t in range(1, 50):
        xb = bytes([0x80]) + bytes(46) + bytes([t]) + bytes(48)
        code = bls.classify_signature(xb)
        cases[xb] = code
    for b, want in cases.items():
        got = L.emu_sig_decode(b, len(b), o, ctypes.byref(inf))
        assert got == bls.classify_signature(b) == want, (b.hex(), got, want)
    codes = set(cases.values())
    assert bls.BLST_POINT_NOT_ON_CURVE in codes and bls.BLST_POINT_NOT_IN_GROUP in codes


def test_key_validate_matches_c_oracle():
    """Device KeyValidate (decompress + phi(P) == -[z^2]P subgroup check) vs the C oracle's definitional
    [r]P == O check, on the reference's cachedKeys (cli/test/utils/cachedKeys.ts:15-26) and on adversarial
    48-byte candidates covering every error class."""
    from oracle import cpu

    L = lib()
    out = ctypes.create_string_buffer(96)
    cands = [bytes.fromhex(h) for h in (
        "8be678633e927aa0435addad5dcd5283fef6110d91362519cd6d43e61f6c017d724fa579cc4b2972134e050b6ba120c0",
        "8e602f8ec17777c22f465f9b4707c2840647790f15f5c33bd8850f274d5c320850105639960ae4effe57aa5dd279bb98")]
    cands += [bytes([0xC0]) + bytes(47), bytes(48), bytes([0x9F]) + bytes([0xFF]) * 47]
    cands += [bytes([0x80 | (t & 0x20)]) + bytes(45) + t.to_bytes(2, "big") for t in range(1, 120)]
    seen = set()
    for c in cands:
        st = L.emu_key_validate(c, len(c), out)
        want = cpu.key_validate(c)
        assert st == want, c.hex()
        seen.add(st)
        if st == 0:
            assert cpu.pk_decode(c) == (0, out.raw)
            assert L.emu_key_validate(out.raw, 96, out) == 0
    assert {0, bls.BLST_BAD_ENCODING, bls.BLST_POINT_NOT_ON_CURVE, bls.BLST_POINT_NOT_IN_GROUP,
            bls.BLST_PK_IS_INFINITY} <= seen


def _r_of_word(w):
    from tests.emu_helpers import r_of_word

    return r_of_word(w)


def test_batch_scalar_word_multiplication():
    """k_common.hpp jac_mul_scalar_word (host copy): [a]P + [b] lambda(P) with lambda = phi on G1 and -psi^2 on
    G2 equals [r]P for r = a + b lambda mod the group order -- both groups use the same r."""
    from tests.emu_helpers import b2g1, g1b, r_of_word

    L = lib()
    L.emu_g1_mul_word.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p]
    L.emu_g2_mul_word.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p]
    r2 = random.Random(91)
    P = bls.g1_mul(bls.G1_GEN, r2.randrange(1, bls.R))
    Q = bls.g2_mul(bls.G2_GEN, r2.randrange(1, bls.R))
    o1, o2 = buf(96), buf(192)
    for w in [0, 1, 2**32 - 1, 2**32, 2**64 - 1, 0x8000000080000000] + [r2.getrandbits(64) for _ in range(6)]:
        r = r_of_word(w, raw=True)
        assert L.emu_g1_mul_word(g1b(P), w, o1) == 1 and b2g1(o1.raw) == bls.g1_mul(P, r), hex(w)
        assert L.emu_g2_mul_word(g2b(Q), w, o2) == 1 and b2g2(o2.raw) == bls.g2_mul(Q, r), hex(w)


def test_bucket_msm_matches_sum_of_scalings():
    """msm.hpp (the k_msm.hip algorithm) against the oracle's sum of r_i P_i: random points and words, r = 1
    words, skipped points, and the exceptional bucket additions (the same point twice, P and -P)."""
    L = lib()
    L.emu_msm.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_char_p, ctypes.c_int,
                          ctypes.c_char_p]
    r2 = random.Random(77)
    base = [bls.g2_mul(bls.G2_GEN, r2.randrange(1, bls.R)) for _ in range(6)]
    cases = [
        (base[:1], [r2.getrandbits(64)], None),
        (base[:1], [0], None),                                   # CoreVerify: r = 1
        (base[:5], [r2.getrandbits(64) for _ in range(5)], None),
        (base[:3] + base[:3], [7, 7, 7, 7, 7, 7], None),         # equal points, equal words: bucket doublings
        (base[:2] + [bls.g2_neg(base[0])], [9, 5, 9], None),     # P and -P with one word: bucket cancellation
        (base, [r2.getrandbits(64) for _ in range(6)], bytes([1, 0, 1, 1, 0, 1])),
        (base[:2], [1, 2], bytes([0, 0])),                       # nothing active: infinity
    ]
    out = buf(192)
    for pts, words, active in cases:
        n = len(pts)
        W = (ctypes.c_uint64 * n)(*words)
        got = L.emu_msm(b"".join(g2b(p) for p in pts), W, active, n, out)
        want = None
        for i, p in enumerate(pts):
            if active is not None and not active[i]:
                continue
            q = bls.g2_mul(p, _r_of_word(words[i]) % bls.R)
            want = q if want is None else bls.g2_add(want, q)
        if want is None:
            assert got == 0
        else:
            assert got == 1 and b2g2(out.raw) == want, (words, active)


def _limbs_of(v, r2):
    """A 14 x 28-bit limb pattern of the integer v: normalized, or with random borrows moved into the lower
    limbs so limbs reach up to 2^29 - 1 (the un-normalized operands fp2_mul_lazy_body accepts)."""
    l = [(v >> (28 * i)) & 0xFFFFFFF for i in range(14)]
    l[13] = v >> (28 * 13)
    if r2.random() < 0.5:
        for i in range(13):
            if l[i + 1] > 0 and r2.random() < 0.7:
                l[i + 1] -= 1
                l[i] += 1 << 28
    assert sum(x << (28 * i) for i, x in enumerate(l)) == v and all(0 <= x < 2**29 for x in l)
    return l


def test_fp2_mul_lazy_reduction_bounds():
    """tower.hpp fp2_mul_lazy_body on raw limbs at the edges of its contract (limbs < 2^29, values < 8p):
    c0 = (a0 b0 - a1 b1) / R and c1 = (a0 b1 + a1 b0) / R mod p, outputs normalized and < 1.06 p."""
    L = lib()
    L.emu_fp2_mul_lazy_limbs.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]
    r2 = random.Random(4242)
    RINV = pow(2**392, -1, P)
    edge = [0, 1, P - 1, P, 2 * P, 8 * P - 1, 8 * P - 2**300, 2**383, 2**384 - 1 if 2**384 - 1 < 8 * P else 8 * P - 1]
    out = (ctypes.c_uint32 * 28)()
    for it in range(3000):
        vals = [r2.choice(edge) if r2.random() < 0.3 else r2.randrange(8 * P) for _ in range(4)]
        limbs = [x for v in vals for x in _limbs_of(v, r2)]
        L.emu_fp2_mul_lazy_limbs((ctypes.c_uint32 * 56)(*limbs), out)
        o = list(out)
        assert all(x < 2**28 for x in o), (vals, o)
        c0 = sum(x << (28 * i) for i, x in enumerate(o[:14]))
        c1 = sum(x << (28 * i) for i, x in enumerate(o[14:]))
        a0, a1, b0, b1 = vals
        assert c0 < 1.06 * P and c1 < 1.06 * P, (vals,)
        assert c0 % P == (a0 * b0 - a1 * b1) * RINV % P, (it, vals)
        assert c1 % P == (a0 * b1 + a1 * b0) * RINV % P, (it, vals)


def test_hash_to_g2_two_lane_split_matches_oracle():
    """k_hash_map / k_hash_clear's split of hash_to_G2 (one SSWU map per lane, then sum and cofactor clearing)
    against the oracle's hash_to_g2 (RFC 9380 BLS12381G2_XMD:SHA-256_SSWU_RO_ with the POP DST)."""
    L = lib()
    out = buf(192)
    for j in range(6):
        m = bytes([j * 37 % 256]) * 32 if j < 3 else random.Random(j).randbytes(32)
        assert L.emu_hash_to_g2_split(m, out) == 1
        assert b2g2(out.raw) == bls.hash_to_g2(m)


def _raw(v):
    return [(v >> (28 * i)) & 0xFFFFFFF if i < 13 else v >> (28 * 13) for i in range(14)]


def _val(l):
    return sum(int(x) << (28 * i) for i, x in enumerate(l))


def test_lacc_fin_and_lazy_operands():
    """gt_wave.hpp's recombination (lacc.hpp lacc_fin: carry pass, integer quotient estimate, one conditional
    subtraction) at the edges of its contract -- up to 15 terms of 2p per side, limb sums at their maxima -- and the
    cooperative squaring's lazy operands (fp_sub_k8: x0 + 8p - x1 unreduced) for values up to 4p, against Python."""
    L = lib()
    r2 = random.Random(515)
    A32 = ctypes.c_uint32 * 14
    out = A32()
    R_INV = pow(2**392, -1, P)
    for trial in range(3000):
        npos, nneg = r2.randint(0, 15), r2.randint(0, 15)
        terms_p = [r2.choice([0, 2 * P, P, r2.randrange(2 * P + 1)]) for _ in range(npos)]
        terms_n = [r2.choice([0, 2 * P, P - 1, r2.randrange(2 * P + 1)]) for _ in range(nneg)]
        pos = [sum(_raw(t)[i] for t in terms_p) for i in range(14)]
        neg = [sum(_raw(t)[i] for t in terms_n) for i in range(14)]
        if trial % 7 == 0:  # limb sums at their maxima: 15 normalized limbs of 2^28 - 1
            pos = [15 * 0xFFFFFFF if i < 13 else 15 * _raw(2 * P)[13] for i in range(14)]
        L.emu_lacc_fin(A32(*pos), A32(*neg), out)
        v = _val(out)
        assert all(x < 2**28 for x in out[:13]) and v <= 2 * P, trial
        assert (v - (_val(pos) - _val(neg))) % P == 0, trial
    for trial in range(2000):
        x0 = r2.choice([0, 4 * P, 2 * P, r2.randrange(4 * P + 1)])
        x1 = r2.choice([0, 4 * P, 2 * P, r2.randrange(4 * P + 1)])
        L.emu_sqr_operands_mul(A32(*_raw(x0)), A32(*_raw(x1)), out)
        v = _val(out)
        assert all(x < 2**28 for x in out[:13]) and v < 2 * P, trial
        assert v % P == (x0 + x1) * (x0 - x1) * R_INV % P, trial


def test_cooperative_g2_addition():
    """g2_coop.hpp g2c_add: the cooperative Jacobian addition (five product phases + five recombinations, operands
    with different Z), phases run lane by lane on the host, against the oracle's affine sum -- generic pairs, points
    outside G2, and the exceptional cases jac_add handles (P = Q, P = -Q, an infinite operand)."""
    L = lib()
    o = buf(192)
    r2 = random.Random(909)
    pts = [bls.g2_mul(bls.G2_GEN, r2.randrange(1, bls.R)) for _ in range(4)]
    while len(pts) < 6:  # points of E2 not in G2
        x = (r2.randrange(P), r2.randrange(P))
        y = bls.f2sqrt(bls.f2add(bls.f2mul(bls.f2sqr(x), x), bls.B2))
        if y:
            pts.append((x, y))
    neg = lambda q: (q[0], bls.f2neg(q[1]))
    cases = [(pts[i], pts[j]) for i in range(6) for j in range(6) if i != j]
    cases += [(q, q) for q in pts] + [(q, neg(q)) for q in pts] + [(None, pts[0]), (pts[1], None), (None, None)]
    for p_, q_ in cases:
        want = bls.g2_add(p_, q_)
        rc = L.emu_g2c_add(g2b(p_) if p_ else bytes(192), int(p_ is None), g2b(q_) if q_ else bytes(192),
                           int(q_ is None), o)
        if want is None:
            assert rc == 0
        else:
            assert rc == 1 and b2g2(o.raw) == want


def test_cooperative_g2_doubling_chain():
    """g2_coop.hpp: the [|z|] chain as the 16-lane groups run it (three product phases + two recombinations per
    doubling, cooperative additions), phases executed lane by lane on the host, against the oracle's [|z|]P -- on G2
    points and on points of E2 outside G2 (the cofactor clearing's inputs)."""
    L = lib()
    o = buf(192)
    r2 = random.Random(808)
    pts = [bls.g2_mul(bls.G2_GEN, r2.randrange(1, bls.R)) for _ in range(3)]
    while len(pts) < 6:  # points of E2 not in G2
        x = (r2.randrange(P), r2.randrange(P))
        y = bls.f2sqrt(bls.f2add(bls.f2mul(bls.f2sqr(x), x), bls.B2))
        if y:
            pts.append((x, y))
    for q in pts:
        assert L.emu_g2c_mul_zabs(g2b(q), o) == 1
        assert b2g2(o.raw) == bls.g2_mul(q, 0xD201000000010000)


def _limbs14(v):
    return [(v >> (28 * i)) & ((1 << 28) - 1) for i in range(13)] + [v >> (28 * 13)]


def _val14(l):
    return sum(x << (28 * i) for i, x in enumerate(l))


def test_fp_lc_edges():
    """fp_lc (fp.hpp): lazily reduced linear combinations at the edges of the contract -- terms of value 0, 1, p - 1,
    p, 2p - 1, 2p and random values <= 2p, with the maximal weight 15 -- are the combination mod p, normalized, below
    1.003 p."""
    import random

    L = lib()
    L.emu_fp_lc_7p8n.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]
    L.emu_fp_lc_weighted.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]
    P = bls.P
    edges = [0, 1, P - 1, P, 2 * P - 1, 2 * P, (1 << 28) - 1]
    rnd = random.Random(11)
    for trial in range(3000):
        pick = lambda: rnd.choice(edges) if rnd.random() < 0.5 else rnd.randrange(0, 2 * P + 1)
        if trial < 4:  # extreme sign patterns: all positives at 2p and negatives at 0, and the reverse
            xs = [2 * P if (k < 7) == (trial % 2 == 0) else 0 for k in range(15)]
        else:
            xs = [pick() for _ in range(15)]
        arr = (ctypes.c_uint32 * 210)(*sum((_limbs14(x) for x in xs), []))
        out = (ctypes.c_uint32 * 14)()
        L.emu_fp_lc_7p8n(arr, out)
        v = _val14(list(out))
        assert all(x < (1 << 28) for x in list(out)[:13]) and v < 1.003 * P
        assert v % P == (sum(xs[:7]) - sum(xs[7:])) % P
        ws = [2, -3, 5, -4, 1]
        ys = xs[:5]
        arr = (ctypes.c_uint32 * 70)(*sum((_limbs14(x) for x in ys), []))
        L.emu_fp_lc_weighted(arr, out)
        v = _val14(list(out))
        assert all(x < (1 << 28) for x in list(out)[:13]) and v < 1.003 * P
        assert v % P == sum(w * y for w, y in zip(ws, ys)) % P


def test_fp2_sqr_operand_contract():
    """fp2_sqr (tower.hpp) on normalized operands of value up to 4p -- the sums the lazy point formulas hand it
    (F_add_sq / fp2_add_norm) -- including a1 - a0 > 2p, where the earlier a0 + 2p - a1 form underflowed: the Montgomery
    square (a0 + a1 u)^2 R^-1, normalized, below 1.05 p."""
    import random

    L = lib()
    L.emu_fp2_sqr_limbs.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]
    P = bls.P
    Rinv = pow(1 << 392, -1, P)
    rnd = random.Random(12)
    edges = [0, 1, P - 1, P, 2 * P, 3 * P + 5, 4 * P - 1, 4 * P]
    for trial in range(2000):
        if trial < 64:
            a0, a1 = edges[trial % 8], edges[trial // 8]
        elif trial < 200:  # the underflow shape: a0 small, a1 near 4p
            a0, a1 = rnd.randrange(0, P // 8), rnd.randrange(3 * P, 4 * P + 1)
        else:
            a0, a1 = rnd.randrange(0, 4 * P + 1), rnd.randrange(0, 4 * P + 1)
        arr = (ctypes.c_uint32 * 28)(*(_limbs14(a0) + _limbs14(a1)))
        out = (ctypes.c_uint32 * 28)()
        L.emu_fp2_sqr_limbs(arr, out)
        c0, c1 = _val14(list(out)[:14]), _val14(list(out)[14:])
        for c in (list(out)[:13], list(out)[14:27]):
            assert all(x < (1 << 28) for x in c)
        assert c0 < 1.05 * P and c1 < 1.05 * P, (trial, c0 / P, c1 / P)
        assert c0 % P == (a0 * a0 - a1 * a1) * Rinv % P, trial
        assert c1 % P == 2 * a0 * a1 * Rinv % P, trial


def test_line_pair_product():
    """The Miller accumulation's chunks of two: f * (l_a * l_b) by line_pair + fp12_mul_by_line2 equals two sparse
    products f * l_a * l_b (tower.hpp), on random Fp12 values and random line coefficients (host build)."""
    import random

    L = lib()
    L.emu_line_pair_check.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    P = bls.P
    rnd = random.Random(21)
    for _ in range(200):
        f = b"".join(rnd.randrange(P).to_bytes(48, "big") for _ in range(12))
        lines = b"".join(rnd.randrange(P).to_bytes(48, "big") for _ in range(12))
        assert L.emu_line_pair_check(f, lines) == 1


def test_fp2_mul_schoolbook_offset_bounds():
    """tower.hpp fp2_mul_sb_body (c0 = Redc(a0 b0 + a1 (16p - b1)), c1 = Redc(a0 b1 + a1 b0)) on raw limbs at the
    edges of the same contract (limbs < 2^29, values < 8p): the Fp2 product / R mod p, normalized, below 1.1 p."""
    L = lib()
    L.emu_fp2_mul_sb_limbs.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]
    r2 = random.Random(4343)
    RINV = pow(2**392, -1, P)
    edge = [0, 1, P - 1, P, 2 * P, 8 * P - 1, 8 * P - 2**300, 2**383]
    out = (ctypes.c_uint32 * 28)()
    for it in range(3000):
        vals = [r2.choice(edge) if r2.random() < 0.3 else r2.randrange(8 * P) for _ in range(4)]
        limbs = [x for v in vals for x in _limbs_of(v, r2)]
        L.emu_fp2_mul_sb_limbs((ctypes.c_uint32 * 56)(*limbs), out)
        o = list(out)
        assert all(x < 2**28 for x in o), (vals, o)
        c0 = sum(x << (28 * i) for i, x in enumerate(o[:14]))
        c1 = sum(x << (28 * i) for i, x in enumerate(o[14:]))
        a0, a1, b0, b1 = vals
        assert c0 < 1.1 * P and c1 < 1.1 * P, (vals,)
        assert c0 % P == (a0 * b0 - a1 * b1) * RINV % P, (it, vals)
        assert c1 % P == (a0 * b1 + a1 * b0) * RINV % P, (it, vals)

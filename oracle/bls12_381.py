"""CPU oracle for the BLS12-381 signature-set verification path -- TEST INFRASTRUCTURE ONLY.

This module is a plain-Python restatement, written from the public specifications, of the
arithmetic that Lodestar's `IBlsVerifier` path delegates to `@chainsafe/bls@7.1.1` ->
`@chainsafe/blst@0.2.4` (pinned at reference `yarn.lock:436-451`; neither package is present
in /root/reference, so their published algorithms are restated here):

* BLS12-381 curve / field constants (ZCash BLS12-381 spec).
* ZCash point (de)serialisation with blst's error classes (`Signature.fromBytes`, used at
  reference `packages/beacon-node/src/chain/bls/maybeBatch.ts:23,36`).
* RFC 9380 hash-to-curve suite `BLS12381G2_XMD:SHA-256_SSWU_RO_` with the Eth2 POP DST.
* Optimal-ate pairing, final exponentiation, CoreVerify (`maybeBatch.ts:34-38`) and the random
  linear-combination batch verification of `verifyMultipleSignatures` (`maybeBatch.ts:17-26`).
* Interop secret keys (reference `packages/state-transition/src/util/interop.ts:19-22`).

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import this
file, and only as the checker.  The product path (lodestar_amd / libblsgpu) never calls it.

Parity pinning: `tests/test_oracle_kat.py` checks this oracle against the reference's own
known-answer data (interop deposit signature, cachedKeys sk->pk, mainnet block signatures,
G2 infinity).
"""
from __future__ import annotations

import hashlib
import hmac

# ---------------------------------------------------------------------------------------------
# Constants
# ---------------------------------------------------------------------------------------------
P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
BLS_X = -0xD201000000010000  # the BLS parameter z (negative)
BLS_X_ABS = 0xD201000000010000

G1_X = 0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB
G1_Y = 0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1
G2_X = (
    0x024AA2B2F08F0A91260805272DC51051C6E47AD4FA403B02B4510B647AE3D1770BAC0326A805BBEFD48056C8C121BDB8,
    0x13E02B6052719F607DACD3A088274F65596BD0D09920B61AB5DA61BBDC7F5049334CF11213945D57E5AC7D055D042B7E,
)
G2_Y = (
    0x0CE5D527727D6E118CC9CDC6DA2E351AADFD9BAA8CBDD3A76D429A695160D12C923AC9CC3BACA289E193548608B82801,
    0x0606C4A02EA734CC32ACD2B02BC28B99CB3E287E85A763AF267492AB572E99AB3F370D275CEC1DA1AAA9075FF05F79BE,
)

# Eth2 proof-of-possession ciphersuite DST (consensus-specs phase0 `bls.Sign`).
DST_POP = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_"

# blst error codes (names as exposed by @chainsafe/blst; numeric values are ours, see include/blsgpu.h)
BLST_SUCCESS = 0
BLST_BAD_ENCODING = 1
BLST_POINT_NOT_ON_CURVE = 2
BLST_POINT_NOT_IN_GROUP = 3
BLST_AGGR_TYPE_MISMATCH = 4
BLST_VERIFY_FAIL = 5
BLST_PK_IS_INFINITY = 6
BLST_BAD_SCALAR = 7
BLST_INVALID_SIZE = 8
ERROR_NAMES = {
    BLST_BAD_ENCODING: "BLST_BAD_ENCODING",
    BLST_POINT_NOT_ON_CURVE: "BLST_POINT_NOT_ON_CURVE",
    BLST_POINT_NOT_IN_GROUP: "BLST_POINT_NOT_IN_GROUP",
    BLST_AGGR_TYPE_MISMATCH: "BLST_AGGR_TYPE_MISMATCH",
    BLST_VERIFY_FAIL: "BLST_VERIFY_FAIL",
    BLST_PK_IS_INFINITY: "BLST_PK_IS_INFINITY",
    BLST_BAD_SCALAR: "BLST_BAD_SCALAR",
    BLST_INVALID_SIZE: "BLST_INVALID_SIZE",
}


class BlstError(Exception):
    """Mirrors @chainsafe/blst's ErrorBLST: message contains 'BLST_ERROR' and the code name."""

    def __init__(self, code: int):
        self.code = code
        super().__init__(f"BLST_ERROR: {ERROR_NAMES[code]}")


# ---------------------------------------------------------------------------------------------
# Instrumentation: count base-field multiplications (mul + sqr) for the roofline op count.
# ---------------------------------------------------------------------------------------------
class _Counter:
    enabled = False
    fp_mul = 0


def count_reset():
    _Counter.fp_mul = 0


def count_enable(on: bool = True):
    _Counter.enabled = on


def count_get() -> int:
    return _Counter.fp_mul


# ---------------------------------------------------------------------------------------------
# Fp
# ---------------------------------------------------------------------------------------------
def fmul(a, b):
    if _Counter.enabled:
        _Counter.fp_mul += 1
    return a * b % P


def finv(a):
    return pow(a, P - 2, P)


def fsqrt(a):
    """Square root in Fp (p = 3 mod 4). Returns None if a is a non-residue."""
    s = pow(a, (P + 1) // 4, P)
    return s if s * s % P == a % P else None


def f_is_square(a):
    return a % P == 0 or pow(a, (P - 1) // 2, P) == 1


# ---------------------------------------------------------------------------------------------
# Fp2 = Fp[u]/(u^2+1); elements are tuples (c0, c1)
# ---------------------------------------------------------------------------------------------
F2_ZERO = (0, 0)
F2_ONE = (1, 0)


def f2(a0, a1=0):
    return (a0 % P, a1 % P)


def f2add(a, b):
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)


def f2sub(a, b):
    return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)


def f2neg(a):
    return ((-a[0]) % P, (-a[1]) % P)


def f2mul(a, b):
    if _Counter.enabled:
        _Counter.fp_mul += 3
    a0, a1 = a
    b0, b1 = b
    return ((a0 * b0 - a1 * b1) % P, (a0 * b1 + a1 * b0) % P)


def f2sqr(a):
    if _Counter.enabled:
        _Counter.fp_mul += 2
    a0, a1 = a
    return ((a0 + a1) * (a0 - a1) % P, 2 * a0 * a1 % P)


def f2muls(a, s):
    """Fp2 times Fp scalar."""
    if _Counter.enabled:
        _Counter.fp_mul += 2
    return (a[0] * s % P, a[1] * s % P)


def f2conj(a):
    return (a[0], (-a[1]) % P)


def f2inv(a):
    n = (a[0] * a[0] + a[1] * a[1]) % P
    ni = finv(n)
    return (a[0] * ni % P, (-a[1]) * ni % P)


def f2_is_zero(a):
    return a[0] % P == 0 and a[1] % P == 0


def f2pow(a, e):
    r = F2_ONE
    while e:
        if e & 1:
            r = f2mul(r, a)
        a = f2sqr(a)
        e >>= 1
    return r


def f2_is_square(a):
    return f_is_square((a[0] * a[0] + a[1] * a[1]) % P)


def f2sqrt(a):
    """Some square root of a in Fp2, or None.  (Which root is irrelevant: callers fix the sign.)"""
    if f2_is_zero(a):
        return F2_ZERO
    a0, a1 = a
    if a1 == 0:
        s = fsqrt(a0)
        if s is not None:
            return (s, 0)
        s = fsqrt((-a0) % P)
        return (0, s)
    n = (a0 * a0 + a1 * a1) % P
    s = fsqrt(n)
    if s is None:
        return None
    inv2 = (P + 1) // 2
    t = (a0 + s) * inv2 % P
    x0 = fsqrt(t)
    if x0 is None:
        t = (a0 - s) * inv2 % P
        x0 = fsqrt(t)
        if x0 is None:
            return None
    x1 = a1 * finv(2 * x0 % P) % P
    r = (x0, x1)
    assert f2sqr(r) == (a0 % P, a1 % P)
    return r


def sgn0_f2(a):
    """RFC 9380 section 4.1 sgn0 for m = 2."""
    s0 = a[0] % 2
    z0 = a[0] == 0
    s1 = a[1] % 2
    return s0 | (z0 & s1)


def f2_lex_largest(a):
    """ZCash sort flag: y is lexicographically largest (compare c1 first, then c0)."""
    half = (P - 1) // 2
    if a[1] != 0:
        return a[1] > half
    return a[0] > half


def f_lex_largest(a):
    return a > (P - 1) // 2


XI = (1, 1)  # u + 1, the Fp6 non-residue


def f2mul_xi(a):
    # (a0 + a1 u)(1 + u) = (a0 - a1) + (a0 + a1) u
    return ((a[0] - a[1]) % P, (a[0] + a[1]) % P)


def f2frob(a):
    return f2conj(a)


# ---------------------------------------------------------------------------------------------
# Fp6 = Fp2[v]/(v^3 - xi), Fp12 = Fp6[w]/(w^2 - v).  Fp6 = (c0,c1,c2); Fp12 = (c0,c1).
# ---------------------------------------------------------------------------------------------
F6_ZERO = (F2_ZERO, F2_ZERO, F2_ZERO)
F6_ONE = (F2_ONE, F2_ZERO, F2_ZERO)
F12_ONE = (F6_ONE, F6_ZERO)


def f6add(a, b):
    return (f2add(a[0], b[0]), f2add(a[1], b[1]), f2add(a[2], b[2]))


def f6sub(a, b):
    return (f2sub(a[0], b[0]), f2sub(a[1], b[1]), f2sub(a[2], b[2]))


def f6neg(a):
    return (f2neg(a[0]), f2neg(a[1]), f2neg(a[2]))


def f6mul(a, b):
    a0, a1, a2 = a
    b0, b1, b2 = b
    t0 = f2mul(a0, b0)
    t1 = f2mul(a1, b1)
    t2 = f2mul(a2, b2)
    c0 = f2add(t0, f2mul_xi(f2sub(f2mul(f2add(a1, a2), f2add(b1, b2)), f2add(t1, t2))))
    c1 = f2add(f2sub(f2mul(f2add(a0, a1), f2add(b0, b1)), f2add(t0, t1)), f2mul_xi(t2))
    c2 = f2add(f2sub(f2mul(f2add(a0, a2), f2add(b0, b2)), f2add(t0, t2)), t1)
    return (c0, c1, c2)


def f6mul_v(a):
    """Multiply by v: (a0 + a1 v + a2 v^2) v = xi a2 + a0 v + a1 v^2."""
    return (f2mul_xi(a[2]), a[0], a[1])


def f6inv(a):
    a0, a1, a2 = a
    t0 = f2sub(f2sqr(a0), f2mul_xi(f2mul(a1, a2)))
    t1 = f2sub(f2mul_xi(f2sqr(a2)), f2mul(a0, a1))
    t2 = f2sub(f2sqr(a1), f2mul(a0, a2))
    d = f2add(f2mul(a0, t0), f2mul_xi(f2add(f2mul(a2, t1), f2mul(a1, t2))))
    di = f2inv(d)
    return (f2mul(t0, di), f2mul(t1, di), f2mul(t2, di))


def f12mul(a, b):
    a0, a1 = a
    b0, b1 = b
    t0 = f6mul(a0, b0)
    t1 = f6mul(a1, b1)
    c1 = f6sub(f6mul(f6add(a0, a1), f6add(b0, b1)), f6add(t0, t1))
    c0 = f6add(t0, f6mul_v(t1))
    return (c0, c1)


def f12sqr(a):
    return f12mul(a, a)


def f12conj(a):
    return (a[0], f6neg(a[1]))


def f12inv(a):
    a0, a1 = a
    t = f6sub(f6mul(a0, a0), f6mul_v(f6mul(a1, a1)))
    ti = f6inv(t)
    return (f6mul(a0, ti), f6neg(f6mul(a1, ti)))


def f12_is_one(a):
    return a == F12_ONE


def f12pow(a, e):
    r = F12_ONE
    while e:
        if e & 1:
            r = f12mul(r, a)
        a = f12sqr(a)
        e >>= 1
    return r


# Frobenius constants, derived from first principles (not transcribed).
def _frob_consts():
    # gamma_{k,j} = xi^{j (p^k - 1)/6}, j = 1..5, for k = 1, 2, 3
    g = {}
    for k in (1, 2, 3):
        for j in range(1, 6):
            g[(k, j)] = f2pow(XI, j * (P**k - 1) // 6)
    return g


_GAMMA = _frob_consts()


def f12frob(a, k=1):
    """a^(p^k).  Element = sum_{i} c_i w^i, c_i in Fp2, with w^i index i = 0..5 where
    c0 = (g0, g2, g4) i.e. w^0, w^2, w^4 and c1 = (g1, g3, g5)."""
    (g0, g2, g4), (g1, g3, g5) = a
    coeffs = [g0, g1, g2, g3, g4, g5]
    out = []
    for i, c in enumerate(coeffs):
        cc = c if k % 2 == 0 else f2conj(c)
        if i:
            cc = f2mul(cc, _GAMMA[(k, i)])
        out.append(cc)
    return ((out[0], out[2], out[4]), (out[1], out[3], out[5]))


# ---------------------------------------------------------------------------------------------
# Generic Fp12 as polynomials mod w^12 - 2 w^6 + 2 (definitional cross-check of the tower)
# ---------------------------------------------------------------------------------------------
def tower_to_poly(a):
    (g0, g2, g4), (g1, g3, g5) = a
    coeffs = [g0, g1, g2, g3, g4, g5]
    poly = [0] * 12
    for k, (x, y) in enumerate(coeffs):  # x + y u, u = w^6 - 1
        poly[k] = (poly[k] + x - y) % P
        poly[k + 6] = (poly[k + 6] + y) % P
    return poly


def poly_mul(a, b):
    prod = [0] * 23
    for i in range(12):
        if a[i] == 0:
            continue
        for j in range(12):
            prod[i + j] += a[i] * b[j]
    # reduce with w^12 = 2 w^6 - 2
    for k in range(22, 11, -1):
        c = prod[k] % P
        if c:
            prod[k] = 0
            prod[k - 6] += 2 * c
            prod[k - 12] -= 2 * c
    return [x % P for x in prod[:12]]


# ---------------------------------------------------------------------------------------------
# Curves. G1: y^2 = x^3 + 4 over Fp.  G2 (twist): y^2 = x^3 + 4(u+1) over Fp2.
# Points are affine tuples or None for infinity.  Jacobian arithmetic for speed.
# ---------------------------------------------------------------------------------------------
B1 = 4
B2 = (4, 4)


class Fp1Ops:
    zero = 0
    one = 1
    add = staticmethod(lambda a, b: (a + b) % P)
    sub = staticmethod(lambda a, b: (a - b) % P)
    mul = staticmethod(fmul)
    sqr = staticmethod(lambda a: fmul(a, a))
    neg = staticmethod(lambda a: (-a) % P)
    inv = staticmethod(finv)
    is_zero = staticmethod(lambda a: a % P == 0)
    b = B1


class Fp2Ops:
    zero = F2_ZERO
    one = F2_ONE
    add = staticmethod(f2add)
    sub = staticmethod(f2sub)
    mul = staticmethod(f2mul)
    sqr = staticmethod(f2sqr)
    neg = staticmethod(f2neg)
    inv = staticmethod(f2inv)
    is_zero = staticmethod(f2_is_zero)
    b = B2


def on_curve(F, pt):
    if pt is None:
        return True
    x, y = pt
    return F.sub(F.sqr(y), F.add(F.mul(F.sqr(x), x), F.b)) == F.zero


def jac_from_affine(F, pt):
    if pt is None:
        return (F.one, F.one, F.zero)
    return (pt[0], pt[1], F.one)


def jac_to_affine(F, J):
    X, Y, Z = J
    if F.is_zero(Z):
        return None
    zi = F.inv(Z)
    zi2 = F.sqr(zi)
    return (F.mul(X, zi2), F.mul(Y, F.mul(zi2, zi)))


def jac_double(F, J):
    X, Y, Z = J
    if F.is_zero(Z):
        return J
    A = F.sqr(X)
    B = F.sqr(Y)
    C = F.sqr(B)
    D = F.sub(F.sqr(F.add(X, B)), F.add(A, C))
    D = F.add(D, D)
    E = F.add(F.add(A, A), A)
    Fv = F.sqr(E)
    X3 = F.sub(Fv, F.add(D, D))
    C8 = F.add(C, C)
    C8 = F.add(C8, C8)
    C8 = F.add(C8, C8)
    Y3 = F.sub(F.mul(E, F.sub(D, X3)), C8)
    Z3 = F.mul(F.add(Y, Y), Z)
    return (X3, Y3, Z3)


def jac_add(F, J1, J2):
    X1, Y1, Z1 = J1
    X2, Y2, Z2 = J2
    if F.is_zero(Z1):
        return J2
    if F.is_zero(Z2):
        return J1
    Z1Z1 = F.sqr(Z1)
    Z2Z2 = F.sqr(Z2)
    U1 = F.mul(X1, Z2Z2)
    U2 = F.mul(X2, Z1Z1)
    S1 = F.mul(Y1, F.mul(Z2, Z2Z2))
    S2 = F.mul(Y2, F.mul(Z1, Z1Z1))
    H = F.sub(U2, U1)
    Rr = F.sub(S2, S1)
    if F.is_zero(H):
        if F.is_zero(Rr):
            return jac_double(F, J1)
        return (F.one, F.one, F.zero)
    H2 = F.sqr(H)
    H3 = F.mul(H, H2)
    U1H2 = F.mul(U1, H2)
    X3 = F.sub(F.sub(F.sqr(Rr), H3), F.add(U1H2, U1H2))
    Y3 = F.sub(F.mul(Rr, F.sub(U1H2, X3)), F.mul(S1, H3))
    Z3 = F.mul(H, F.mul(Z1, Z2))
    return (X3, Y3, Z3)


def jac_neg(F, J):
    return (J[0], F.neg(J[1]), J[2])


def jac_mul(F, J, k):
    if k < 0:
        return jac_mul(F, jac_neg(F, J), -k)
    Rj = (F.one, F.one, F.zero)
    for bit in bin(k)[2:] if k else "":
        Rj = jac_double(F, Rj)
        if bit == "1":
            Rj = jac_add(F, Rj, J)
    return Rj


def g1_mul(pt, k):
    return jac_to_affine(Fp1Ops, jac_mul(Fp1Ops, jac_from_affine(Fp1Ops, pt), k))


def g2_mul(pt, k):
    return jac_to_affine(Fp2Ops, jac_mul(Fp2Ops, jac_from_affine(Fp2Ops, pt), k))


def g1_add(a, b):
    return jac_to_affine(Fp1Ops, jac_add(Fp1Ops, jac_from_affine(Fp1Ops, a), jac_from_affine(Fp1Ops, b)))


def g2_add(a, b):
    return jac_to_affine(Fp2Ops, jac_add(Fp2Ops, jac_from_affine(Fp2Ops, a), jac_from_affine(Fp2Ops, b)))


def g1_neg(a):
    return None if a is None else (a[0], (-a[1]) % P)


def g2_neg(a):
    return None if a is None else (a[0], f2neg(a[1]))


G1_GEN = (G1_X, G1_Y)
G2_GEN = (G2_X, G2_Y)


# psi endomorphism on the twist: psi(x, y) = (conj(x) * PSI_X, conj(y) * PSI_Y)
PSI_X = f2inv(f2pow(XI, (P - 1) // 3))
PSI_Y = f2inv(f2pow(XI, (P - 1) // 2))


def g2_psi(pt):
    if pt is None:
        return None
    return (f2mul(f2conj(pt[0]), PSI_X), f2mul(f2conj(pt[1]), PSI_Y))


def g2_in_subgroup_def(pt):
    """Definitional check [r]P == O."""
    return pt is None or g2_mul(pt, R) is None


def g2_in_subgroup_psi(pt):
    """Scott (eprint 2021/1130): P in G2 iff psi(P) == [z]P.  Product algorithm."""
    if pt is None:
        return True
    return g2_psi(pt) == g2_mul(pt, BLS_X)


# ---------------------------------------------------------------------------------------------
# Serialisation (ZCash format)
# ---------------------------------------------------------------------------------------------
def fp_to_bytes(a):
    return a.to_bytes(48, "big")


def g1_compress(pt):
    if pt is None:
        return bytes([0xC0]) + bytes(47)
    x, y = pt
    b = bytearray(fp_to_bytes(x))
    b[0] |= 0x80
    if f_lex_largest(y):
        b[0] |= 0x20
    return bytes(b)


def g1_serialize(pt):
    if pt is None:
        return bytes([0x40]) + bytes(95)
    return fp_to_bytes(pt[0]) + fp_to_bytes(pt[1])


def g2_compress(pt):
    if pt is None:
        return bytes([0xC0]) + bytes(95)
    x, y = pt
    b = bytearray(fp_to_bytes(x[1]) + fp_to_bytes(x[0]))
    b[0] |= 0x80
    if f2_lex_largest(y):
        b[0] |= 0x20
    return bytes(b)


def g2_serialize(pt):
    if pt is None:
        return bytes([0x40]) + bytes(191)
    x, y = pt
    return fp_to_bytes(x[1]) + fp_to_bytes(x[0]) + fp_to_bytes(y[1]) + fp_to_bytes(y[0])


def g1_decompress(b):
    """blst POINTonE1_Uncompress_Z semantics; raises BlstError."""
    if len(b) != 48:
        raise BlstError(BLST_INVALID_SIZE)
    b0 = b[0]
    if not b0 & 0x80:
        raise BlstError(BLST_BAD_ENCODING)
    if b0 & 0x40:
        if (b0 & 0x3F) == 0 and not any(b[1:]):
            return None
        raise BlstError(BLST_BAD_ENCODING)
    x = int.from_bytes(bytes([b0 & 0x1F]) + b[1:], "big")
    if x >= P:
        raise BlstError(BLST_BAD_ENCODING)
    y = fsqrt((x * x * x + B1) % P)
    if y is None:
        raise BlstError(BLST_POINT_NOT_ON_CURVE)
    if f_lex_largest(y) != bool(b0 & 0x20):
        y = (-y) % P
    return (x, y)


def g1_deserialize(b):
    """Affine 96-byte (uncompressed) or 48-byte compressed, blst_p1_deserialize semantics."""
    if len(b) == 48:
        return g1_decompress(b)
    if len(b) != 96:
        raise BlstError(BLST_INVALID_SIZE)
    b0 = b[0]
    if b0 & 0x80:
        raise BlstError(BLST_BAD_ENCODING)
    if b0 & 0x40:
        if (b0 & 0x3F) == 0 and not any(b[1:]):
            return None
        raise BlstError(BLST_BAD_ENCODING)
    if b0 & 0x20:
        raise BlstError(BLST_BAD_ENCODING)
    x = int.from_bytes(b[:48], "big")
    y = int.from_bytes(b[48:], "big")
    if x >= P or y >= P:
        raise BlstError(BLST_BAD_ENCODING)
    if not on_curve(Fp1Ops, (x, y)):
        raise BlstError(BLST_POINT_NOT_ON_CURVE)
    return (x, y)


def g2_decompress_raw(b):
    """Returns (point, err).  Size must already be 96.  blst POINTonE2_Uncompress_Z semantics."""
    b0 = b[0]
    if not b0 & 0x80:
        return None, BLST_BAD_ENCODING
    if b0 & 0x40:
        if (b0 & 0x3F) == 0 and not any(b[1:]):
            return None, BLST_SUCCESS
        return None, BLST_BAD_ENCODING
    x1 = int.from_bytes(bytes([b0 & 0x1F]) + b[1:48], "big")
    x0 = int.from_bytes(b[48:96], "big")
    if x1 >= P or x0 >= P:
        return None, BLST_BAD_ENCODING
    x = (x0, x1)
    y = f2sqrt(f2add(f2mul(f2sqr(x), x), B2))
    if y is None:
        return None, BLST_POINT_NOT_ON_CURVE
    if f2_lex_largest(y) != bool(b0 & 0x20):
        y = f2neg(y)
    return (x, y), BLST_SUCCESS


def g2_deserialize_raw(b):
    """192-byte uncompressed affine.  blst POINTonE2_Deserialize_Z semantics."""
    b0 = b[0]
    if b0 & 0x80:
        return None, BLST_BAD_ENCODING
    if b0 & 0x40:
        if (b0 & 0x3F) == 0 and not any(b[1:]):
            return None, BLST_SUCCESS
        return None, BLST_BAD_ENCODING
    if b0 & 0x20:
        return None, BLST_BAD_ENCODING
    x1 = int.from_bytes(b[0:48], "big")
    x0 = int.from_bytes(b[48:96], "big")
    y1 = int.from_bytes(b[96:144], "big")
    y0 = int.from_bytes(b[144:192], "big")
    if max(x0, x1, y0, y1) >= P:
        return None, BLST_BAD_ENCODING
    pt = ((x0, x1), (y0, y1))
    if not on_curve(Fp2Ops, pt):
        return None, BLST_POINT_NOT_ON_CURVE
    return pt, BLST_SUCCESS


def signature_from_bytes(b, validate=True, subgroup=g2_in_subgroup_psi):
    """`bls.Signature.fromBytes(bytes, CoordType.affine, validate)` (maybeBatch.ts:23,36).
    Raises BlstError; returns affine point or None (infinity)."""
    b = bytes(b)
    if len(b) == 96:
        pt, err = g2_decompress_raw(b)
    elif len(b) == 192:
        pt, err = g2_deserialize_raw(b)
    else:
        raise BlstError(BLST_INVALID_SIZE)
    if err:
        raise BlstError(err)
    if validate and not subgroup(pt):
        raise BlstError(BLST_POINT_NOT_IN_GROUP)
    return pt


def classify_signature(b):
    """Status code for a signature byte string (0 = ok)."""
    try:
        signature_from_bytes(b)
        return BLST_SUCCESS
    except BlstError as e:
        return e.code


# ---------------------------------------------------------------------------------------------
# Hash to G2 (RFC 9380, BLS12381G2_XMD:SHA-256_SSWU_RO_)
# ---------------------------------------------------------------------------------------------
def expand_message_xmd(msg: bytes, dst: bytes, len_in_bytes: int) -> bytes:
    b_in_bytes, s_in_bytes = 32, 64
    ell = (len_in_bytes + b_in_bytes - 1) // b_in_bytes
    assert ell <= 255 and len(dst) <= 255
    dst_prime = dst + bytes([len(dst)])
    z_pad = bytes(s_in_bytes)
    l_i_b = len_in_bytes.to_bytes(2, "big")
    b0 = hashlib.sha256(z_pad + msg + l_i_b + b"\x00" + dst_prime).digest()
    bi = hashlib.sha256(b0 + b"\x01" + dst_prime).digest()
    out = bi
    for i in range(2, ell + 1):
        bi = hashlib.sha256(bytes(x ^ y for x, y in zip(b0, bi)) + bytes([i]) + dst_prime).digest()
        out += bi
    return out[:len_in_bytes]


def hash_to_field_fp2(msg: bytes, count: int, dst: bytes = DST_POP):
    L = 64
    ub = expand_message_xmd(msg, dst, count * 2 * L)
    out = []
    for i in range(count):
        e = []
        for j in range(2):
            off = L * (j + i * 2)
            e.append(int.from_bytes(ub[off : off + L], "big") % P)
        out.append((e[0], e[1]))
    return out


# SSWU parameters for the 3-isogenous curve E2': y^2 = x^3 + A' x + B'
SSWU_A = (0, 240)
SSWU_B = (1012, 1012)
SSWU_Z = ((-2) % P, (-1) % P)


def map_to_curve_sswu(u):
    """RFC 9380 section 6.6.2 simplified SWU (non-constant-time restatement)."""
    A, B, Z = SSWU_A, SSWU_B, SSWU_Z
    u2 = f2sqr(u)
    Zu2 = f2mul(Z, u2)
    tv = f2add(f2sqr(Zu2), Zu2)  # Z^2 u^4 + Z u^2
    if f2_is_zero(tv):
        x1 = f2mul(B, f2inv(f2mul(Z, A)))
    else:
        x1 = f2mul(f2mul(f2neg(B), f2inv(A)), f2add(F2_ONE, f2inv(tv)))
    gx1 = f2add(f2mul(f2add(f2sqr(x1), A), x1), B)
    if f2_is_square(gx1):
        x, y = x1, f2sqrt(gx1)
    else:
        x2 = f2mul(Zu2, x1)
        gx2 = f2add(f2mul(f2add(f2sqr(x2), A), x2), B)
        x, y = x2, f2sqrt(gx2)
    if sgn0_f2(u) != sgn0_f2(y):
        y = f2neg(y)
    return (x, y)


def _h(s):
    return int(s, 16)


# 3-isogeny map E2' -> E2 (RFC 9380 Appendix E.3).  Validated by tests (image on curve,
# homomorphism) and end-to-end by the interop deposit KAT.
_PM = P
ISO3_XNUM = [
    (_h("5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97d6"),
     _h("5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97d6")),
    (0, _h("11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71a")),
    (_h("11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71e"),
     _h("8ab05f8bdd54cde190937e76bc3e447cc27c3d6fbd7063fcd104635a790520c0a395554e5c6aaaa9354ffffffffe38d")),
    (_h("171d6541fa38ccfaed6dea691f5fb614cb14b4e7f4e810aa22d6108f142b85757098e38d0f671c7188e2aaaaaaaa5ed1"), 0),
]
ISO3_XDEN = [
    (0, _PM - 72),
    (12, _PM - 12),
    (1, 0),
]
ISO3_YNUM = [
    (_h("1530477c7ab4113b59a4c18b076d11930f7da5d4a07f649bf54439d87d27e500fc8c25ebf8c92f6812cfc71c71c6d706"),
     _h("1530477c7ab4113b59a4c18b076d11930f7da5d4a07f649bf54439d87d27e500fc8c25ebf8c92f6812cfc71c71c6d706")),
    (0, _h("5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97be")),
    (_h("11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71c"),
     _h("8ab05f8bdd54cde190937e76bc3e447cc27c3d6fbd7063fcd104635a790520c0a395554e5c6aaaa9354ffffffffe38f")),
    (_h("124c9ad43b6cf79bfbf7043de3811ad0761b0f37a1e26286b0e977c69aa274524e79097a56dc4bd9e1b371c71c718b10"), 0),
]
ISO3_YDEN = [
    (_PM - 432, _PM - 432),
    (0, _PM - 216),
    (18, _PM - 18),
    (1, 0),
]


def _poly_eval(coeffs, x):
    acc = F2_ZERO
    for c in reversed(coeffs):
        acc = f2add(f2mul(acc, x), c)
    return acc


def iso3_map(pt):
    if pt is None:
        return None
    x, y = pt
    xn = _poly_eval(ISO3_XNUM, x)
    xd = _poly_eval(ISO3_XDEN, x)
    yn = _poly_eval(ISO3_YNUM, x)
    yd = _poly_eval(ISO3_YDEN, x)
    if f2_is_zero(xd) or f2_is_zero(yd):
        return None
    return (f2mul(xn, f2inv(xd)), f2mul(y, f2mul(yn, f2inv(yd))))


def clear_cofactor_g2(pt):
    """RFC 9380 Appendix G.3 (Budroni-Pintore), equal to multiplication by h_eff."""
    F = Fp2Ops
    Pj = jac_from_affine(F, pt)
    c1 = BLS_X
    t1 = jac_mul(F, Pj, c1)
    t2 = jac_from_affine(F, g2_psi(jac_to_affine(F, Pj)))
    t3 = jac_double(F, Pj)
    t3 = jac_from_affine(F, g2_psi(g2_psi(jac_to_affine(F, t3))))
    t3 = jac_add(F, t3, jac_neg(F, t2))
    t2 = jac_add(F, t1, t2)
    t2 = jac_mul(F, t2, c1)
    t3 = jac_add(F, t3, t2)
    t3 = jac_add(F, t3, jac_neg(F, t1))
    Q = jac_add(F, t3, jac_neg(F, Pj))
    return jac_to_affine(F, Q)


H_EFF_G2 = _h(
    "bc69f08f2ee75b3584c6a0ea91b352888e2a8e9145ad7689986ff031508ffe1329c2f178731db956d82bf015d1212b02ec0ec69d7477c1ae954cbc06689f6a359894c0adebbf6b4e8020005aaa95551"
)


def hash_to_g2(msg: bytes, dst: bytes = DST_POP):
    u0, u1 = hash_to_field_fp2(msg, 2, dst)
    q0 = iso3_map(map_to_curve_sswu(u0))
    q1 = iso3_map(map_to_curve_sswu(u1))
    return clear_cofactor_g2(g2_add(q0, q1))


# ---------------------------------------------------------------------------------------------
# Pairing
# ---------------------------------------------------------------------------------------------
def _line_to_f12(a0, a1, b1):
    """Sparse line  a0 + a1 v + b1 v w  (positions c0.c0, c0.c1, c1.c1)."""
    return ((a0, a1, F2_ZERO), (F2_ZERO, b1, F2_ZERO))


def miller_loop_affine(Pp, Qp):
    """Definitional Miller loop f_{|z|,Q}(P) with affine lines on the twist, each line scaled by
    w^3 (an Fp4 element, killed by the final exponentiation).  Returns f (not conjugated)."""
    if Pp is None or Qp is None:
        return F12_ONE
    xP, yP = Pp
    f = F12_ONE
    T = Qp
    bits = bin(BLS_X_ABS)[3:]
    for bit in bits:
        x, y = T
        lam = f2mul(f2muls(f2sqr(x), 3), f2inv(f2add(y, y)))
        line = _line_to_f12(f2sub(f2mul(lam, x), y), f2neg(f2muls(lam, xP)), (yP, 0))
        f = f12mul(f12sqr(f), line)
        x3 = f2sub(f2sqr(lam), f2add(x, x))
        T = (x3, f2sub(f2mul(lam, f2sub(x, x3)), y))
        if bit == "1":
            x, y = T
            xq, yq = Qp
            lam = f2mul(f2sub(yq, y), f2inv(f2sub(xq, x)))
            line = _line_to_f12(f2sub(f2mul(lam, x), y), f2neg(f2muls(lam, xP)), (yP, 0))
            f = f12mul(f, line)
            x3 = f2sub(f2sub(f2sqr(lam), x), xq)
            T = (x3, f2sub(f2mul(lam, f2sub(x, x3)), y))
    return f


# --- projective Miller loop: the exact algorithm the HIP kernels implement -------------------
B2_3 = f2muls(B2, 3)  # 3 b'


def dbl_step(T, xP, yP):
    """Homogeneous projective doubling on E2 with line (Costello-Lange-Naehrig 2010 / Aranha et al.
    2010 formulas).  Line = (E - B) + (3 X^2 xP) v + (-H yP) v w."""
    X, Y, Z = T
    A = f2mul(X, Y)
    A = f2muls(A, (P + 1) // 2)  # X Y / 2  (counted as a multiplication by a constant)
    Bv = f2sqr(Y)
    C = f2sqr(Z)
    E = f2mul(B2_3, C)
    Fv = f2add(f2add(E, E), E)
    G = f2muls(f2add(Bv, Fv), (P + 1) // 2)
    H = f2sub(f2sqr(f2add(Y, Z)), f2add(Bv, C))
    J = f2sqr(X)
    E2 = f2sqr(E)
    X3 = f2mul(A, f2sub(Bv, Fv))
    Y3 = f2sub(f2sqr(G), f2add(f2add(E2, E2), E2))
    Z3 = f2mul(Bv, H)
    l0 = f2sub(E, Bv)
    l1 = f2muls(f2add(f2add(J, J), J), xP)
    l4 = f2muls(f2neg(H), yP)
    return (X3, Y3, Z3), (l0, l1, l4)


def add_step(T, Q, xP, yP):
    """Mixed addition T + Q (Q affine) with line.  Line = (theta x2 - lambda y2)
    + (-theta xP) v + (lambda yP) v w."""
    X, Y, Z = T
    x2, y2 = Q
    theta = f2sub(Y, f2mul(y2, Z))
    lam = f2sub(X, f2mul(x2, Z))
    C = f2sqr(theta)
    D = f2sqr(lam)
    E = f2mul(lam, D)
    Fv = f2mul(Z, C)
    G = f2mul(X, D)
    H = f2sub(f2add(E, Fv), f2add(G, G))
    X3 = f2mul(lam, H)
    Y3 = f2sub(f2mul(theta, f2sub(G, H)), f2mul(Y, E))
    Z3 = f2mul(Z, E)
    l0 = f2sub(f2mul(theta, x2), f2mul(lam, y2))
    l1 = f2muls(f2neg(theta), xP)
    l4 = f2muls(lam, yP)
    return (X3, Y3, Z3), (l0, l1, l4)


def f12_mul_by_014(f, l0, l1, l4):
    return f12mul(f, _line_to_f12(l0, l1, l4))


def miller_loop_proj(Pp, Qp):
    """f_{|z|,Q}(P) with projective steps (no conjugation).  Same as the device algorithm."""
    if Pp is None or Qp is None:
        return F12_ONE
    xP, yP = Pp
    T = (Qp[0], Qp[1], F2_ONE)
    f = F12_ONE
    first = True
    for bit in bin(BLS_X_ABS)[3:]:
        if not first:
            f = f12sqr(f)
        T, (l0, l1, l4) = dbl_step(T, xP, yP)
        f = f12_mul_by_014(f, l0, l1, l4)
        first = False
        if bit == "1":
            T, (l0, l1, l4) = add_step(T, Qp, xP, yP)
            f = f12_mul_by_014(f, l0, l1, l4)
    return f


def miller_loop(Pp, Qp):
    """Optimal ate Miller loop value for the negative BLS parameter: conj(f_{|z|,Q}(P))."""
    return f12conj(miller_loop_proj(Pp, Qp))


def final_exp_def(f):
    """Definitional final exponentiation f^((p^12-1)/r)."""
    f1 = f12mul(f12conj(f), f12inv(f))  # p^6 - 1
    f2_ = f12mul(f12frob(f1, 2), f1)  # p^2 + 1
    return f12pow(f2_, (P**4 - P**2 + 1) // R)


def _cyc_exp_x(f):
    """f^z for z = BLS_X < 0 in the cyclotomic subgroup: conj(f^|z|)."""
    return f12conj(f12pow(f, BLS_X_ABS))


def final_exp(f):
    """Final exponentiation used by the device: easy part, then the hard part as
    3 (p^4 - p^2 + 1)/r = (z-1)^2 (z+p) (z^2+p^2-1) + 3.  Returns e^3 (same 'is one' answer,
    gcd(3, r) = 1)."""
    f1 = f12mul(f12conj(f), f12inv(f))
    m = f12mul(f12frob(f1, 2), f1)
    # y0 = m^((z-1)^2) = (m^(z-1))^(z-1);  m^(z-1) = m^z * conj(m)
    t = f12mul(_cyc_exp_x(m), f12conj(m))
    t = f12mul(_cyc_exp_x(t), f12conj(t))
    # t^(z+p)
    t = f12mul(_cyc_exp_x(t), f12frob(t, 1))
    # t^(z^2 + p^2 - 1)
    t = f12mul(f12mul(_cyc_exp_x(_cyc_exp_x(t)), f12frob(t, 2)), f12conj(t))
    # times m^3
    return f12mul(t, f12mul(f12sqr(m), m))


def pairing(Pp, Qp):
    return final_exp(miller_loop(Pp, Qp))


# ---------------------------------------------------------------------------------------------
# Keys, signing, verification
# ---------------------------------------------------------------------------------------------
def sk_to_pk(sk: int):
    return g1_mul(G1_GEN, sk)


def sign(sk: int, msg: bytes):
    return g2_mul(hash_to_g2(msg), sk)


def core_verify(pk, msg: bytes, sig) -> bool:
    """e(pk, H(m)) * e(-g1, sig) == 1 (blst core_verify, hash_or_encode = hash)."""
    if pk is None:
        raise BlstError(BLST_PK_IS_INFINITY)
    H = hash_to_g2(msg)
    f = f12mul(miller_loop(pk, H), miller_loop(g1_neg(G1_GEN), sig))
    return f12_is_one(final_exp(f))


class SplitMix64:
    """Deterministic batch randomness for comparison runs.  Production uses a CSPRNG."""

    def __init__(self, seed: int):
        self.state = seed & 0xFFFFFFFFFFFFFFFF

    def next(self) -> int:
        self.state = (self.state + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
        z = self.state
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
        return z ^ (z >> 31)

    def nonzero(self) -> int:
        while True:
            v = self.next()
            if v:
                return v


def batch_verify(sets, scalars) -> bool:
    """verifyMultipleSignatures: prod e(r_i pk_i, H(m_i)) * e(-g1, sum r_i sig_i) == 1.
    `sets` = [(pk_affine, msg, sig_affine)] with signatures already deserialised+validated."""
    f = F12_ONE
    S = None
    for (pk, msg, sig), r in zip(sets, scalars):
        if pk is None:
            raise BlstError(BLST_PK_IS_INFINITY)
        H = hash_to_g2(msg)
        f = f12mul(f, miller_loop(g1_mul(pk, r), H))
        S = g2_add(S, g2_mul(sig, r))
    f = f12mul(f, miller_loop(g1_neg(G1_GEN), S))
    return f12_is_one(final_exp(f))


def verify_signature_sets_maybe_batch(sets, rng: SplitMix64 | None = None):
    """Restates `verifySignatureSetsMaybeBatch` (reference maybeBatch.ts:16-39).
    sets = [(pk_affine, msg_bytes, sig_bytes)].  Raises BlstError / ValueError like the reference."""
    if len(sets) >= 2:
        des = [(pk, msg, signature_from_bytes(sig)) for pk, msg, sig in sets]
        rng = rng or SplitMix64(0x4C4F444553544152)
        scalars = [rng.nonzero() for _ in des]
        return batch_verify(des, scalars)
    if len(sets) == 0:
        raise ValueError("Empty signature set")
    pk, msg, sig = sets[0]
    return core_verify(pk, msg, signature_from_bytes(sig))


def key_validate(pk_bytes: bytes):
    """PublicKey.fromBytes(pk, validate=true) (reference state-transition/src/block/processDeposit.ts:56-64,
    beacon-node/test/spec/general/bls.ts:121-124): decode (48 or 96 bytes), reject the identity and points
    outside G1 (definitional [r]P == O).  Returns the affine point or raises BlstError."""
    pt = g1_deserialize(bytes(pk_bytes))
    if pt is None:
        raise BlstError(BLST_PK_IS_INFINITY)
    if g1_mul(pt, R) is not None:
        raise BlstError(BLST_POINT_NOT_IN_GROUP)
    return pt


def fast_aggregate_verify(pks_bytes, msg: bytes, sig_bytes: bytes) -> bool:
    """The spec runner's fast_aggregate_verify (reference beacon-node/test/spec/general/bls.ts:117-127):
    Signature.fromBytes(validate) . verifyAggregate(PublicKey.fromBytes(validate) of each key); any error
    -> false (EMPTY_AGGREGATE_ARRAY included)."""
    try:
        sig = signature_from_bytes(sig_bytes)
        pks = [key_validate(p) for p in pks_bytes]
        if not pks:
            raise ValueError("EMPTY_AGGREGATE_ARRAY")
        return core_verify(aggregate_pubkeys(pks), msg, sig)
    except (BlstError, ValueError):
        return False


G1_INFINITY_COMPRESSED = bytes([0xC0]) + bytes(47)
G2_INFINITY_COMPRESSED = bytes([0xC0]) + bytes(95)


def eth_fast_aggregate_verify(pks_bytes, msg: bytes, sig_bytes: bytes) -> bool:
    """eth_fast_aggregate_verify (reference spec/general/bls.ts:93-112): no keys + infinity signature ->
    true; an infinity key -> false; otherwise fast_aggregate_verify."""
    if not pks_bytes and bytes(sig_bytes) == G2_INFINITY_COMPRESSED:
        return True
    if any(bytes(p) == G1_INFINITY_COMPRESSED for p in pks_bytes):
        return False
    return fast_aggregate_verify(pks_bytes, msg, sig_bytes)


def aggregate_pubkeys(pks):
    """bls.PublicKey.aggregate (reference chain/bls/utils.ts:11)."""
    if len(pks) == 0:
        raise ValueError("EMPTY_AGGREGATE_ARRAY")
    acc = (1, 1, 0)
    for pk in pks:
        acc = jac_add(Fp1Ops, acc, jac_from_affine(Fp1Ops, pk))
    return jac_to_affine(Fp1Ops, acc)


def interop_secret_key(index: int) -> int:
    """reference packages/state-transition/src/util/interop.ts:19-22:
    sk = bytesToBigInt(sha256(intToBytes(index, 32))) mod r  -- intToBytes is little-endian
    (packages/utils/src/bytes.ts:20-47) and bytesToBigInt is little-endian as well."""
    h = hashlib.sha256(index.to_bytes(32, "little")).digest()
    return int.from_bytes(h, "little") % R


def keygen_ietf(ikm: bytes, key_info: bytes = b"") -> int:
    """IETF BLS KeyGen (draft-irtf-cfrg-bls-signature-04+), as blst_keygen."""
    salt = b"BLS-SIG-KEYGEN-SALT-"
    L = 48
    sk = 0
    while sk == 0:
        salt = hashlib.sha256(salt).digest()
        prk = hmac.new(salt, ikm + b"\x00", hashlib.sha256).digest()
        okm = b""
        t = b""
        i = 1
        info = key_info + L.to_bytes(2, "big")
        while len(okm) < L:
            t = hmac.new(prk, t + info + bytes([i]), hashlib.sha256).digest()
            okm += t
            i += 1
        sk = int.from_bytes(okm[:L], "big") % R
    return sk

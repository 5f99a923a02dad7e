// Per-element operations of the verification path, shared by the HIP kernels (kernels.hip).
// Byte formats follow the ZCash BLS12-381 encoding used by blst / @chainsafe/blst.
#pragma once
#include "hash_to_curve.hpp"
#include "pairing.hpp"

// Status codes: blst error names as thrown by @chainsafe/blst (see include/blsgpu.h)
enum {
  BLS_OK = 0,
  BLS_BAD_ENCODING = 1,
  BLS_POINT_NOT_ON_CURVE = 2,
  BLS_POINT_NOT_IN_GROUP = 3,
  BLS_AGGR_TYPE_MISMATCH = 4,
  BLS_VERIFY_FAIL = 5,
  BLS_PK_IS_INFINITY = 6,
  BLS_BAD_SCALAR = 7,
  BLS_INVALID_SIZE = 8,
  BLS_EMPTY_AGGREGATE = 9,
  BLS_EMPTY_SET = 10,
  BLS_DEVICE_ERROR = 11,
};

BLS_HD bool bytes_all_zero(const uint8_t* b, int n) {
  uint32_t o = 0;
  for (int i = 0; i < n; i++) o |= b[i];
  return o == 0;
}

// Deserialize a G2 signature: 96-byte compressed or 192-byte uncompressed (blst_p2_deserialize /
// POINTonE2_Uncompress_Z semantics) -- everything of Signature.fromBytes but the subgroup check.
// Returns a status; on success `inf` tells whether the point is the identity.
BLS_HDNI int sig_decode_point(const uint8_t* b, uint32_t len, g2a& out, bool& inf) {
  inf = false;
  if (len != 96 && len != 192) return BLS_INVALID_SIZE;
  const uint8_t b0 = b[0];
  const bool compressed = (b0 & 0x80) != 0;
  if (compressed != (len == 96)) return BLS_BAD_ENCODING;
  if (b0 & 0x40) {
    if ((b0 & 0x3f) == 0 && bytes_all_zero(b + 1, (int)len - 1)) {
      inf = true;
      return BLS_OK;
    }
    return BLS_BAD_ENCODING;
  }
  fp x1, x0;
  bool ok1 = fp_from_be48_plain(b, x1, 0x1f);
  bool ok0 = fp_from_be48_plain(b + 48, x0, 0xff);
  if (compressed) {
    if (!ok1 || !ok0) return BLS_BAD_ENCODING;
    g2a p;
    p.x = fp2_make(fp_to_mont(x0), fp_to_mont(x1));
    fp2 rhs = fp2_add(fp2_mul(fp2_sqr(p.x), p.x), FP2_B2);
    fp2 y;
    if (!fp2_sqrt(rhs, y)) return BLS_POINT_NOT_ON_CURVE;
    // sort flag: y lexicographically largest (compare c1, then c0)
    fp2 yp = fp2_plain(y);
    bool c1z = fp_is_zero(yp.c1);
    bool largest = c1z ? fp_plain_gt_half(yp.c0) : fp_plain_gt_half(yp.c1);
    bool want = (b0 & 0x20) != 0;
    p.y = fp2_select(largest != want, fp2_neg(y), y);
    out = p;
  } else {
    if (b0 & 0x20) return BLS_BAD_ENCODING;
    fp y1, y0;
    bool ok3 = fp_from_be48_plain(b + 96, y1, 0xff);
    bool ok2 = fp_from_be48_plain(b + 144, y0, 0xff);
    if (!ok1 || !ok0 || !ok2 || !ok3) return BLS_BAD_ENCODING;
    g2a p;
    p.x = fp2_make(fp_to_mont(x0), fp_to_mont(x1));
    p.y = fp2_make(fp_to_mont(y0), fp_to_mont(y1));
    if (!g2_on_curve(p)) return BLS_POINT_NOT_ON_CURVE;
    out = p;
  }
  return BLS_OK;
}
// ... then subgroup-check it (`validate = true`, maybeBatch.ts:23,36)
BLS_HDNI int sig_decode(const uint8_t* b, uint32_t len, g2a& out, bool& inf) {
  const int st = sig_decode_point(b, len, out, inf);
  if (st != BLS_OK || inf) return st;
  return g2_in_subgroup(out) ? BLS_OK : BLS_POINT_NOT_IN_GROUP;
}

// Deserialize a trusted 96-byte uncompressed affine G1 public key (blst_p1_deserialize semantics,
// as used by the pool worker: PublicKey.fromBytes(pk, CoordType.affine), worker.ts:110-116).
BLS_HDNI int pk_decode96(const uint8_t* b, g1a& out, bool& inf) {
  inf = false;
  const uint8_t b0 = b[0];
  if (b0 & 0x80) return BLS_BAD_ENCODING;
  if (b0 & 0x40) {
    if ((b0 & 0x3f) == 0 && bytes_all_zero(b + 1, 95)) {
      inf = true;
      return BLS_OK;
    }
    return BLS_BAD_ENCODING;
  }
  if (b0 & 0x20) return BLS_BAD_ENCODING;
  fp x, y;
  bool okx = fp_from_be48_plain(b, x, 0xff);
  bool oky = fp_from_be48_plain(b + 48, y, 0xff);
  if (!okx || !oky) return BLS_BAD_ENCODING;
  out.x = fp_to_mont(x);
  out.y = fp_to_mont(y);
  if (!g1_on_curve(out)) return BLS_POINT_NOT_ON_CURVE;
  return BLS_OK;
}

// G1 subgroup check for KeyValidate: phi(P) == -[z^2]P with phi(x, y) = (beta x, y) (Scott, eprint
// 2021/1130; the definitional [r]P == O is the oracle's, tests/test_emu_logic.py compares the two).
BLS_HDNI bool g1_in_subgroup(const g1a& p) {
  g1j P = jac_from_aff(p);
  g1j z2P = jac_mul_zabs(jac_mul_zabs(P));  // [z^2]P (z^2 > 0)
  g1j phi = P;
  phi.x = fp_mul(p.x, G1_BETA);
  return jac_eq(phi, jac_neg(z2P));
}

// Decompress a 48-byte G1 encoding (blst POINTonE1_Uncompress semantics); no subgroup check.
BLS_HDNI int pk_decode48(const uint8_t* b, g1a& out, bool& inf) {
  inf = false;
  const uint8_t b0 = b[0];
  if (!(b0 & 0x80)) return BLS_BAD_ENCODING;
  if (b0 & 0x40) {
    if ((b0 & 0x3f) == 0 && bytes_all_zero(b + 1, 47)) {
      inf = true;
      return BLS_OK;
    }
    return BLS_BAD_ENCODING;
  }
  fp x;
  if (!fp_from_be48_plain(b, x, 0x1f)) return BLS_BAD_ENCODING;
  out.x = fp_to_mont(x);
  const fp rhs = fp_add(fp_mul(fp_sqr(out.x), out.x), FP_B1);
  fp y = fp_mul(rhs, fp_pow_p34(rhs));  // rhs^((p+1)/4)
  if (!fp_eq(fp_sqr(y), rhs)) return BLS_POINT_NOT_ON_CURVE;
  const bool largest = fp_plain_gt_half(fp_from_mont(y));
  if (largest != ((b0 & 0x20) != 0)) y = fp_neg(y);
  out.y = y;
  return BLS_OK;
}

// KeyValidate (PublicKey.fromBytes(pk, validate = true): processDeposit.ts:56-64, spec bls.ts:33-42):
// 48- or 96-byte encoding, not the identity, in G1.
BLS_HDNI int pk_key_validate(const uint8_t* b, uint32_t len, g1a& out) {
  bool inf = false;
  int st;
  if (len == 48)
    st = pk_decode48(b, out, inf);
  else if (len == 96)
    st = pk_decode96(b, out, inf);
  else
    return BLS_INVALID_SIZE;
  if (st != BLS_OK) return st;
  if (inf) return BLS_PK_IS_INFINITY;
  return g1_in_subgroup(out) ? BLS_OK : BLS_POINT_NOT_IN_GROUP;
}

BLS_HD void fp_to_be48(const fp& mont, uint8_t* b) { fp_to_be48_plain(fp_from_mont(mont), b); }

BLS_HD void g2a_to_be192(const g2a& p, uint8_t* b) {
  fp_to_be48(p.x.c1, b);
  fp_to_be48(p.x.c0, b + 48);
  fp_to_be48(p.y.c1, b + 96);
  fp_to_be48(p.y.c0, b + 144);
}
BLS_HD void g1a_to_be96(const g1a& p, uint8_t* b) {
  fp_to_be48(p.x, b);
  fp_to_be48(p.y, b + 48);
}

// ZCash compressed encoding of an affine G1 point (not infinity)
BLS_HD void g1a_compress(const g1a& p, uint8_t* b) {
  fp_to_be48(p.x, b);
  const bool largest = fp_plain_gt_half(fp_from_mont(p.y));
  b[0] |= 0x80 | (largest ? 0x20 : 0);
}

// ZCash compressed encoding of an affine G2 point (not infinity)
BLS_HD void g2a_compress(const g2a& p, uint8_t* b) {
  fp_to_be48(p.x.c1, b);
  fp_to_be48(p.x.c0, b + 48);
  fp2 yp = fp2_plain(p.y);
  bool c1z = fp_is_zero(yp.c1);
  bool largest = c1z ? fp_plain_gt_half(yp.c0) : fp_plain_gt_half(yp.c1);
  b[0] |= 0x80 | (largest ? 0x20 : 0);
}

// RFC 9380 hash_to_curve for BLS12381G2_XMD:SHA-256_SSWU_RO_ with the Eth2 POP DST
// "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_" -- the hash used inside blst's core_verify /
// mul_n_aggregate for every `verifySignatureSets` set (reference maybeBatch.ts:17-38).
// Specialised for 32-byte messages (Lodestar signing roots, reference ISignatureSet.signingRoot).
#pragma once
#include "curve.hpp"

// ------------------------------------------------------------------------------------ SHA-256
BLS_CONST uint32_t SHA256_K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
BLS_CONST uint32_t SHA256_IV[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                   0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};

BLS_HD uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

// One compression of a 16-word (big-endian words) block into the state.  State and block travel by value as
// aggregates of <= 16 dwords, which the AMDGPU calling convention passes and returns in VGPRs; the schedule is fully
// unrolled, so w[] is register-resident too (no scratch frame).
struct sha_st {
  uint32_t h[8];
};
struct sha_blk {
  uint32_t w[16];
};
BLS_HDNI sha_st sha256_block(sha_st st, sha_blk blk) {
  uint32_t a = st.h[0], b = st.h[1], c = st.h[2], d = st.h[3], e = st.h[4], f = st.h[5], g = st.h[6], h = st.h[7];
#pragma unroll
  for (int i = 0; i < 64; i++) {
    uint32_t wi;
    if (i < 16) {
      wi = blk.w[i];
    } else {
      const uint32_t w15 = blk.w[(i - 15) & 15], w2 = blk.w[(i - 2) & 15];
      const uint32_t s0 = rotr32(w15, 7) ^ rotr32(w15, 18) ^ (w15 >> 3);
      const uint32_t s1 = rotr32(w2, 17) ^ rotr32(w2, 19) ^ (w2 >> 10);
      wi = blk.w[i & 15] + s0 + blk.w[(i - 7) & 15] + s1;
      blk.w[i & 15] = wi;
    }
    const uint32_t S1 = rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25);
    const uint32_t ch = (e & f) ^ (~e & g);
    const uint32_t t1 = h + S1 + ch + SHA256_K[i] + wi;
    const uint32_t S0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22);
    const uint32_t maj = (a & b) ^ (a & c) ^ (b & c);
    const uint32_t t2 = S0 + maj;
    h = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
  }
  st.h[0] += a;
  st.h[1] += b;
  st.h[2] += c;
  st.h[3] += d;
  st.h[4] += e;
  st.h[5] += f;
  st.h[6] += g;
  st.h[7] += h;
  return st;
}

// Byte-wise writer into a word buffer (big-endian words); every call site has a constant position
BLS_HD void put_byte(uint32_t* words, int pos, uint32_t byte) {
  words[pos >> 2] |= (byte & 0xffu) << (24 - 8 * (pos & 3));
}
BLS_INL sha_blk sha_blk_of(const uint32_t* w) {
  sha_blk b;
#pragma unroll
  for (int i = 0; i < 16; i++) b.w[i] = w[i];
  return b;
}

// expand_message_xmd(msg(32), DST, 256) -> 64 words (big-endian).  Inlined with every loop unrolled: all buffer
// positions are constants, so the buffers live in registers.
BLS_INL void expand_message_xmd_32(const uint8_t msg[32], uint32_t out[64]) {
  // b0 = H(Z_pad(64) || msg || I2OSP(256,2) || 0x00 || DST || len(DST))
  // Z_pad fills exactly the first block: start from the state after compressing a zero block.
  sha_st st;
#pragma unroll
  for (int i = 0; i < 8; i++) st.h[i] = SHA256_IV[i];
  sha_blk zero;
#pragma unroll
  for (int i = 0; i < 16; i++) zero.w[i] = 0;
  st = sha256_block(st, zero);
  // remaining bytes: msg(32) || 0x01 0x00 || 0x00 || DST(43) || 43  = 79 bytes, total 143
  uint32_t buf[32];
#pragma unroll
  for (int i = 0; i < 32; i++) buf[i] = 0;
#pragma unroll
  for (int i = 0; i < 32; i++) put_byte(buf, i, msg[i]);
  put_byte(buf, 32, 0x01);
  put_byte(buf, 33, 0x00);
  put_byte(buf, 34, 0x00);
#pragma unroll
  for (int i = 0; i < BLS_DST_LEN; i++) put_byte(buf, 35 + i, BLS_DST[i]);
  put_byte(buf, 35 + BLS_DST_LEN, BLS_DST_LEN);
  put_byte(buf, 36 + BLS_DST_LEN, 0x80);
  // total length 143 bytes = 1144 bits, in the last 8 bytes of the second block of buf
  buf[31] = 143u * 8u;
  st = sha256_block(st, sha_blk_of(buf));
  st = sha256_block(st, sha_blk_of(buf + 16));
  const sha_st b0 = st;
  // b_i = H((b0 ^ b_{i-1}) || I2OSP(i,1) || DST || len(DST)) : 32 + 1 + 44 = 77 bytes -> 2 blocks
  sha_st prev;
#pragma unroll
  for (int i = 0; i < 8; i++) prev.h[i] = 0;
#pragma unroll
  for (int idx = 1; idx <= 8; idx++) {
    uint32_t bb[32];
#pragma unroll
    for (int i = 0; i < 32; i++) bb[i] = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) bb[i] = b0.h[i] ^ prev.h[i];
    put_byte(bb, 32, (uint32_t)idx);
#pragma unroll
    for (int i = 0; i < BLS_DST_LEN; i++) put_byte(bb, 33 + i, BLS_DST[i]);
    put_byte(bb, 33 + BLS_DST_LEN, BLS_DST_LEN);
    put_byte(bb, 34 + BLS_DST_LEN, 0x80);
    bb[31] = 77u * 8u;
    sha_st s2;
#pragma unroll
    for (int i = 0; i < 8; i++) s2.h[i] = SHA256_IV[i];
    s2 = sha256_block(s2, sha_blk_of(bb));
    s2 = sha256_block(s2, sha_blk_of(bb + 16));
#pragma unroll
    for (int i = 0; i < 8; i++) out[(idx - 1) * 8 + i] = s2.h[i];
    prev = s2;
  }
}

// 64 big-endian bytes (as 16 big-endian words) -> element of Fp in Montgomery form
BLS_HD fp fp_from_be64_words(const uint32_t* w) {
  // value = sum_j byte_j ... ; build 28-bit limbs of the 512-bit integer: 19 limbs (532 bits)
  uint32_t lim[19];
#pragma unroll
  for (int i = 0; i < 19; i++) lim[i] = 0;
#pragma unroll
  for (int k = 0; k < 16; k++) {  // word k (from least significant)
    uint32_t v = w[15 - k];
    int bit = 32 * k;
    int li = bit / BLS_LB, off = bit % BLS_LB;
    lim[li] |= (v << off) & BLS_MASK;
    if (li + 1 < 19) lim[li + 1] |= (off == 0) ? (v >> BLS_LB) : ((v >> (BLS_LB - off)) & BLS_MASK);
    if (off > 0 && li + 2 < 19 && (32 - (BLS_LB - off)) > BLS_LB) lim[li + 2] |= v >> (2 * BLS_LB - off);
  }
  fp lo, hi;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) lo.l[i] = lim[i];
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) hi.l[i] = (i < 5) ? lim[BLS_NL + i] : 0;
  // Mont(x) = x R = lo R + hi 2^392 R;  mont_mul(lo, R^2) = lo R;  mont_mul(hi, R^3) = hi R^2 = hi 2^392 R
  return fp_add(fp_mul(lo, FP_R2), fp_mul(hi, FP_R3));
}

// hash_to_field(msg, 2) -> u0, u1 in Fp2
BLS_INL void hash_to_field_fp2x2(const uint8_t msg[32], fp2& u0, fp2& u1) {
  uint32_t ub[64];
  expand_message_xmd_32(msg, ub);
  u0.c0 = fp_from_be64_words(ub + 0);
  u0.c1 = fp_from_be64_words(ub + 16);
  u1.c0 = fp_from_be64_words(ub + 32);
  u1.c1 = fp_from_be64_words(ub + 48);
}

// ----------------------------------------------------------------------------- sqrt helpers
// Given a in Fp2 and s = a square root of N(a) (in Fp), return a square root of a (if a is a square).
BLS_INL fp2 fp2_sqrt_with_normroot(const fp2& a, const fp& s) {
  fp t = fp_half(fp_add(a.c0, s));
  fp t_alt = fp_half(fp_sub(a.c0, s));
  t = fp_select(fp_is_zero(t), t_alt, t);
  fp y = fp_pow_p34(t);
  fp x0 = fp_mul(t, y);
  fp a1y2 = fp_half(fp_mul(a.c1, y));
  bool res_case = fp_eq(fp_sqr(x0), t);
  fp2 r;
  r.c0 = fp_select(res_case, x0, a1y2);
  r.c1 = fp_select(res_case, a1y2, fp_neg(x0));
  return r;
}

// canonical plain (non-Montgomery) copy for sign decisions
BLS_HD fp2 fp2_plain(const fp2& a) { return fp2_make(fp_from_mont(a.c0), fp_from_mont(a.c1)); }

// ----------------------------------------------------------------------------- SSWU + iso3
// map_to_curve_simple_swu on E2': y^2 = x^3 + A'x + B'.  `tv_inv` = inv0(Z^2 u^4 + Z u^2) supplied by
// the caller (batched with the other map's inversion).
BLS_INL g2a sswu_map(const fp2& u, const fp2& Zu2, const fp2& tv, const fp2& tv_inv) {
  fp2 x1 = fp2_mul(SSWU_MINUS_B_OVER_A, fp2_add(fp2_one(), tv_inv));
  x1 = fp2_select(fp2_is_zero(tv), SSWU_B_OVER_ZA, x1);
  fp2 gx1 = fp2_add(fp2_mul(fp2_add(fp2_sqr(x1), SSWU_A), x1), SSWU_B);
  fp2 x2 = fp2_mul(Zu2, x1);
  fp2 gx2 = fp2_add(fp2_mul(fp2_add(fp2_sqr(x2), SSWU_A), x2), SSWU_B);
  fp n1 = fp2_norm(gx1);
  fp s1 = fp_mul(n1, fp_pow_p34(n1));
  bool sq1 = fp_eq(fp_sqr(s1), n1);
  fp nu = fp2_norm(u);
  fp s2 = fp_mul(fp_mul(SSWU_C125, s1), fp_mul(fp_sqr(nu), nu));
  fp2 g = fp2_select(sq1, gx1, gx2);
  fp2 x = fp2_select(sq1, x1, x2);
  fp s = fp_select(sq1, s1, s2);
  fp2 y = fp2_sqrt_with_normroot(g, s);
  fp2 up = fp2_plain(u);
  fp2 yp = fp2_plain(y);
  uint32_t su = fp2_sgn0_plain(up.c0, up.c1);
  uint32_t sy = fp2_sgn0_plain(yp.c0, yp.c1);
  y = fp2_select(su != sy, fp2_neg(y), y);
  g2a r;
  r.x = x;
  r.y = y;
  return r;
}

// 3-isogeny E2' -> E2 producing a Jacobian point (no inversion):
//   x = Nx/Dx, y = y' Ny/Dy  ->  Z = Dx Dy, X = Nx Dx Dy^2, Y = y' Ny Dx^3 Dy^2
BLS_INL g2j iso3_map_jac(const g2a& p) {
  const fp2& x = p.x;
  fp2 x2 = fp2_sqr(x);
  fp2 x3 = fp2_mul(x2, x);
  fp2 Nx = fp2_add(fp2_add(fp2_mul(ISO_XNUM_3, x3), fp2_mul(ISO_XNUM_2, x2)), fp2_add(fp2_mul(ISO_XNUM_1, x), ISO_XNUM_0));
  fp2 Dx = fp2_add(fp2_add(x2, fp2_mul(ISO_XDEN_1, x)), ISO_XDEN_0);  // leading coeff 1
  fp2 Ny = fp2_add(fp2_add(fp2_mul(ISO_YNUM_3, x3), fp2_mul(ISO_YNUM_2, x2)), fp2_add(fp2_mul(ISO_YNUM_1, x), ISO_YNUM_0));
  fp2 Dy = fp2_add(fp2_add(x3, fp2_mul(ISO_YDEN_2, x2)), fp2_add(fp2_mul(ISO_YDEN_1, x), ISO_YDEN_0));
  g2j r;
  fp2 DxDy = fp2_mul(Dx, Dy);
  r.z = DxDy;
  r.x = fp2_mul(fp2_mul(Nx, Dy), DxDy);
  fp2 Dx2 = fp2_sqr(Dx);
  r.y = fp2_mul(fp2_mul(fp2_mul(p.y, Ny), fp2_mul(Dx2, Dx)), fp2_sqr(Dy));
  // degenerate denominators (x is a kernel point): image is infinity
  if (fp2_is_zero(DxDy)) r = jac_infinity<fp2>();
  return r;
}

// RFC 9380 G.3: h_eff * P via psi (Budroni-Pintore)
BLS_HDNI g2j clear_cofactor_g2(const g2j& P) {
  g2j t1 = jac_neg(jac_mul_zabs(P));  // [z]P
  g2j t2 = g2_psi(P);
  g2j t3 = g2_psi2(jac_dbl(P));
  t3 = jac_add(t3, jac_neg(t2));
  t2 = jac_add(t1, t2);
  t2 = jac_neg(jac_mul_zabs(t2));
  t3 = jac_add(t3, t2);
  t3 = jac_add(t3, jac_neg(t1));
  return jac_add(t3, jac_neg(P));
}

// clear_cofactor_g2 with its intermediate points in three caller-provided slots (SoA memory in k_hash_clear)
// instead of registers, reordered so that only the accumulator is live across each [|z|] chain:
//   A = [|z|]P,   C = psi^2(2P) - psi(P) + A - P,   D = [|z|](A - psi(P)),   h_eff P = C + D
// (clear_cofactor_g2's t3 + t2 - t1 - P with t1 = -A, t2 = D, t3 = psi^2(2P) - psi(P)).  Slot 0 holds P on entry;
// slots 1 and 2 are overwritten.  Slot 1 may be slot 0 itself (P is in registers before slot 1 is written).  Over
// any G2 field type F (fp2, or the lane-pair fp2x of fp2x.hpp).
template <class F, class Ld, class St>
BLS_INL jac<F> clear_cofactor_slots(Ld ld, St st) {
  const jac<F> A = jac_mul_zabs_ld<F>([&] { return ld(0); });
  {
    const jac<F> P = ld(0);
    const jac<F> psiP = g2_psi(P);
    st(1, jac_add(A, jac_neg(psiP)));
    st(2, jac_add(jac_add(g2_psi2(jac_dbl(P)), jac_neg(psiP)), jac_add(A, jac_neg(P))));
  }
  const jac<F> D = jac_mul_zabs_ld<F>([&] { return ld(1); });
  return jac_add(D, ld(2));
}
template <class Ld, class St>
BLS_INL g2j clear_cofactor_g2_slots(Ld ld, St st) {
  return clear_cofactor_slots<fp2>(ld, st);
}

// hash_to_G2 in two halves around the one inversion of the two maps, so a kernel can batch that inversion over
// many messages (k_hash.hip + k_inv.hip):
//   prep:   u0, u1 = hash_to_field(msg); Zu2_j = Z u_j^2; tv_j = Zu2_j^2 + Zu2_j; d = a0 a1 (a_j = tv_j, or 1
//           when tv_j = 0 -- then inv0(tv_j) = 0, RFC 9380 inv0); d != 0
//   finish: given d^-1, inv0(tv_j) = d^-1 a_{1-j}, the two SSWU maps, the isogeny, the sum, cofactor clearing.
struct h2c_prep {
  fp2 u0, u1, Zu2_0, Zu2_1, tv0, tv1, d;
};
BLS_INL void hash_to_g2_prep(const uint8_t msg[32], h2c_prep& h) {
  hash_to_field_fp2x2(msg, h.u0, h.u1);
  h.Zu2_0 = fp2_mul(SSWU_Z, fp2_sqr(h.u0));
  h.Zu2_1 = fp2_mul(SSWU_Z, fp2_sqr(h.u1));
  h.tv0 = fp2_add(fp2_sqr(h.Zu2_0), h.Zu2_0);
  h.tv1 = fp2_add(fp2_sqr(h.Zu2_1), h.Zu2_1);
  const fp2 a0 = fp2_select(fp2_is_zero(h.tv0), fp2_one(), h.tv0);
  const fp2 a1 = fp2_select(fp2_is_zero(h.tv1), fp2_one(), h.tv1);
  h.d = fp2_mul(a0, a1);
}
// One of the two maps (j = 0, 1) of the finish step: iso3(SSWU(u_j)) as a Jacobian point.  The pipeline runs the
// two maps of a message on two lanes (k_hash_map), then sums and clears the cofactor (k_hash_clear).
BLS_INL g2j hash_to_g2_map_j(const h2c_prep& h, const fp2& dinv, int j) {
  const bool z0 = fp2_is_zero(h.tv0), z1 = fp2_is_zero(h.tv1);
  const fp2 a_other = j == 0 ? fp2_select(z1, fp2_one(), h.tv1) : fp2_select(z0, fp2_one(), h.tv0);
  const bool zj = j == 0 ? z0 : z1;
  const fp2 inv = fp2_select(zj, fp2_zero(), fp2_mul(dinv, a_other));
  // select the operands, then ONE call: lanes j = 0 and 1 of a wave run the same instruction stream
  const bool j0 = j == 0;
  const g2a q = sswu_map(fp2_select(j0, h.u0, h.u1), fp2_select(j0, h.Zu2_0, h.Zu2_1), fp2_select(j0, h.tv0, h.tv1), inv);
  return iso3_map_jac(q);
}

BLS_HDNI g2j hash_to_g2_finish(const h2c_prep& h, const fp2& dinv) {
  const bool z0 = fp2_is_zero(h.tv0), z1 = fp2_is_zero(h.tv1);
  const fp2 a0 = fp2_select(z0, fp2_one(), h.tv0);
  const fp2 a1 = fp2_select(z1, fp2_one(), h.tv1);
  const fp2 inv0 = fp2_select(z0, fp2_zero(), fp2_mul(dinv, a1));
  const fp2 inv1 = fp2_select(z1, fp2_zero(), fp2_mul(dinv, a0));
  g2a q0 = sswu_map(h.u0, h.Zu2_0, h.tv0, inv0);
  g2a q1 = sswu_map(h.u1, h.Zu2_1, h.tv1, inv1);
  g2j Q = jac_add(iso3_map_jac(q0), iso3_map_jac(q1));
  return clear_cofactor_g2(Q);
}

// hash_to_G2(msg) -> Jacobian point (caller converts to affine)
BLS_HDNI g2j hash_to_g2_jac(const uint8_t msg[32]) {
  h2c_prep h;
  hash_to_g2_prep(msg, h);
  return hash_to_g2_finish(h, fp2_inv(h.d));
}

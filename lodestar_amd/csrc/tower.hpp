// Extension tower of BLS12-381:  Fp2 = Fp[u]/(u^2+1),  Fp6 = Fp2[v]/(v^3-(u+1)),  Fp12 = Fp6[w]/(w^2-v).
// Same tower as the oracle (oracle/bls12_381.py) and as the ZCash/IETF BLS12-381 descriptions.
#pragma once
#include "fp.hpp"

struct fp6 {
  fp2 c0, c1, c2;
};
struct fp12 {
  fp6 c0, c1;
};

// ---------------------------------------------------------------------------------------------- Fp2
BLS_HD fp2 fp2_make(const fp& a, const fp& b) {
  fp2 r;
  r.c0 = a;
  r.c1 = b;
  return r;
}
BLS_HD fp2 fp2_zero() { return fp2_make(fp_zero(), fp_zero()); }
BLS_HD fp2 fp2_one() { return fp2_make(FP_ONE, fp_zero()); }
BLS_FN fp2 fp2_add(const fp2& a, const fp2& b) { return fp2_make(fp_add(a.c0, b.c0), fp_add(a.c1, b.c1)); }
BLS_FN fp2 fp2_sub(const fp2& a, const fp2& b) { return fp2_make(fp_sub(a.c0, b.c0), fp_sub(a.c1, b.c1)); }
BLS_HD fp2 fp2_neg(const fp2& a) { return fp2_make(fp_neg(a.c0), fp_neg(a.c1)); }
BLS_HD fp2 fp2_dbl(const fp2& a) { return fp2_make(fp_dbl(a.c0), fp_dbl(a.c1)); }
BLS_HD fp2 fp2_half(const fp2& a) { return fp2_make(fp_half(a.c0), fp_half(a.c1)); }
BLS_HD fp2 fp2_conj(const fp2& a) { return fp2_make(a.c0, fp_neg(a.c1)); }
BLS_HD fp2 fp2_add_nr(const fp2& a, const fp2& b) { return fp2_make(fp_add_nr(a.c0, b.c0), fp_add_nr(a.c1, b.c1)); }
// carries propagated, no reduction: the operand-side sum an Fp2 squaring takes (normalized, value <= a + b <= 4p)
BLS_HD fp2 fp2_add_norm(const fp2& a, const fp2& b) { return fp2_make(fp_add_norm(a.c0, b.c0), fp_add_norm(a.c1, b.c1)); }

// 64 p^2 in 28 limbs of 28 bits: the multiple of p added to a0 b0 - a1 b1 in fp2_mul_lazy_body so the c0 column sum
// stays a non-negative integer for inputs < 8p (a1 b1 < 64 p^2)
BLS_CONST uint32_t FP2_LAZY_OFS[2 * BLS_NL] = {
    0xc638e40, 0x8000071, 0xbaac9aa, 0xc75d8e0, 0xf5f3b5a, 0xd8844f3, 0x58b0ce0, 0x9c6dd0c, 0xfe47b4f, 0x681259a,
    0x16a1c24, 0x1eca4ba, 0x7218617, 0x475a186, 0x25e3bc0, 0x4c524cc, 0x7729bbd, 0x8b3f45b, 0x2f41429, 0x924d27a,
    0xd19b967, 0x439c11a, 0x8b72439, 0x8bc97a7, 0x49e3aa8, 0xd7f1d2f, 0xde92e30, 0x0000a90};

// Fp2 product with lazy reduction: ONE Montgomery reduction per output coefficient, the three half-products
// (a0 b0, a1 b1, (a0 + a1)(b0 + b1), column sums only) interleaved column by column:
//   c0 = Redc(a0 b0 - a1 b1 + 64 p^2),   c1 = Redc((a0 + a1)(b0 + b1) - a0 b0 - a1 b1)
// 5 x 196 = 980 v_mad_u64_u32 instead of 3 x 392, and five independent MAD chains per column instead of one.
// Inputs: limbs < 2^29 (normalized values or one fp_add_nr level), values < 8p.  Column bounds: t0, t1 < 14 * 2^58,
// t2 < 14 * 2^60 (the limb sums a0_i + a1_i < 2^30 are not normalized); t2 - t0 - t1 is exactly the cross-term
// column sum(a0_i b1_j + a1_i b0_j) >= 0; t0 - t1 + ofs may be negative, so c0 runs on a signed accumulator with
// arithmetic shifts (|acc0| < 2^63).  Outputs: normalized limbs, values < 1.06 p.
BLS_INL fp2 fp2_mul_lazy_body(const fp& a0, const fp& a1, const fp& b0, const fp& b1) {
  uint32_t s[BLS_NL], u[BLS_NL], m0[BLS_NL], m1[BLS_NL];
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) {
    s[i] = a0.l[i] + a1.l[i];
    u[i] = b0.l[i] + b1.l[i];
  }
  int64_t acc0 = 0;
  uint64_t acc1 = 0;
  fp2 r;
#pragma unroll
  for (int k = 0; k < 2 * BLS_NL - 1; k++) {
    const int lo = k < BLS_NL ? 0 : k - BLS_NL + 1, hi = k < BLS_NL ? k : BLS_NL - 1;
    uint64_t t0 = 0, t1 = 0, t2 = 0;
#pragma unroll
    for (int i = lo; i <= hi; i++) {
      t0 += (uint64_t)a0.l[i] * b0.l[k - i];
      t1 += (uint64_t)a1.l[i] * b1.l[k - i];
      t2 += (uint64_t)s[i] * u[k - i];
    }
    acc0 += (int64_t)(t0 - t1) + (int64_t)FP2_LAZY_OFS[k];
    acc1 += t2 - t0 - t1;
    const int mhi = k < BLS_NL ? k - 1 : BLS_NL - 1;
#pragma unroll
    for (int i = lo; i <= mhi; i++) {
      acc0 += (int64_t)((uint64_t)m0[i] * FP_P.l[k - i]);
      acc1 += (uint64_t)m1[i] * FP_P.l[k - i];
    }
    if (k < BLS_NL) {
      const uint32_t q0 = ((uint32_t)acc0 * BLS_N0INV) & BLS_MASK, q1 = ((uint32_t)acc1 * BLS_N0INV) & BLS_MASK;
      m0[k] = q0;
      m1[k] = q1;
      acc0 += (int64_t)((uint64_t)q0 * FP_P.l[0]);
      acc1 += (uint64_t)q1 * FP_P.l[0];
    } else {
      r.c0.l[k - BLS_NL] = (uint32_t)acc0 & BLS_MASK;
      r.c1.l[k - BLS_NL] = (uint32_t)acc1 & BLS_MASK;
    }
    acc0 >>= BLS_LB;  // arithmetic: the low 28 bits are zero (k < 14) or emitted
    acc1 >>= BLS_LB;
  }
  r.c0.l[BLS_NL - 1] = (uint32_t)(acc0 + (int64_t)FP2_LAZY_OFS[2 * BLS_NL - 1]);
  r.c1.l[BLS_NL - 1] = (uint32_t)acc1;
  return r;
}

// 16p with limbs 0-12 borrowed up into [2^29, 2^30): 16p - b has no negative limb for b with limbs < 2^29 and a top
// limb below 0x1a010e (values < 8p, normalized or one fp_add_nr level)
BLS_CONST fp FP_16P_K = {{0x3ffaaab0, 0x3efffffc, 0x3ffffb9c, 0x3ffeb150, 0x3241eabc, 0x30f6b0f3, 0x36730d27, 0x338512bc,
                          0x3774b84c, 0x3bacd761, 0x3a7b6431, 0x369a4b18, 0x3ea397fb, 0x001a010e}};
// Fp2 product as two schoolbook column sums straight into the two Montgomery accumulators, no Karatsuba
// recombination: c0 = Redc(a0 b0 + a1 (16p - b1)) (= a0 b0 - a1 b1 mod p), c1 = Redc(a0 b1 + a1 b0).  784 + 392
// v_mad_u64_u32 against the lazy body's 980, but no 64-bit column subtractions (with their carry hazards), no signed
// accumulator and no operand sums: fewer instruction slots and registers per product.  Inputs as fp2_mul_lazy_body
// (limbs < 2^29, values < 8p); column bound 14 (2^58 + 2^59) + 14 * 2^56 + 2^36 < 2^64; outputs normalized, < 1.1 p.
BLS_INL fp2 fp2_mul_sb_body(const fp& a0, const fp& a1, const fp& b0, const fp& b1) {
  uint32_t nb[BLS_NL], m0[BLS_NL], m1[BLS_NL];
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) nb[i] = FP_16P_K.l[i] - b1.l[i];
  uint64_t acc0 = 0, acc1 = 0;
  fp2 r;
#pragma unroll
  for (int k = 0; k < 2 * BLS_NL - 1; k++) {
    const int lo = k < BLS_NL ? 0 : k - BLS_NL + 1, hi = k < BLS_NL ? k : BLS_NL - 1;
#pragma unroll
    for (int i = lo; i <= hi; i++) {
      acc0 += (uint64_t)a0.l[i] * b0.l[k - i];
      acc1 += (uint64_t)a0.l[i] * b1.l[k - i];
      acc0 += (uint64_t)a1.l[i] * nb[k - i];
      acc1 += (uint64_t)a1.l[i] * b0.l[k - i];
    }
    const int mhi = k < BLS_NL ? k - 1 : BLS_NL - 1;
#pragma unroll
    for (int i = lo; i <= mhi; i++) {
      acc0 += (uint64_t)m0[i] * FP_P.l[k - i];
      acc1 += (uint64_t)m1[i] * FP_P.l[k - i];
    }
    if (k < BLS_NL) {
      const uint32_t q0 = ((uint32_t)acc0 * BLS_N0INV) & BLS_MASK, q1 = ((uint32_t)acc1 * BLS_N0INV) & BLS_MASK;
      m0[k] = q0;
      m1[k] = q1;
      acc0 += (uint64_t)q0 * FP_P.l[0];
      acc1 += (uint64_t)q1 * FP_P.l[0];
    } else {
      r.c0.l[k - BLS_NL] = (uint32_t)acc0 & BLS_MASK;
      r.c1.l[k - BLS_NL] = (uint32_t)acc1 & BLS_MASK;
    }
    acc0 >>= BLS_LB;
    acc1 >>= BLS_LB;
  }
  r.c0.l[BLS_NL - 1] = (uint32_t)acc0;
  r.c1.l[BLS_NL - 1] = (uint32_t)acc1;
  return r;
}
#ifndef BLS_FP2_SB
#define BLS_FP2_SB 1
#endif
#if BLS_FP2_SB
#define fp2_mul_body_sel fp2_mul_sb_body
#else
#define fp2_mul_body_sel fp2_mul_lazy_body
#endif

// Fp2 squaring (complex method): c0 = (a0 + a1)(a0 - a1), c1 = 2 a0 a1 -- two independent products.  Input:
// normalized limbs, values <= 4p (stored values, or fp2_add_norm of two); a0 - a1 goes to the product as
// a0 + 8p - a1 (fp_sub_k8, no reduction), so an input above 2p never underflows.  Outputs < 1.05 p.
BLS_INL fp2 fp2_sqr_body(const fp2& a) {
  const fp c0 = fp_mul_body(fp_add_nr(a.c0, a.c1), fp_sub_k8(a.c0, a.c1));
  const fp c1 = fp_mul_body(fp_add_nr(a.c0, a.c0), a.c1);
  return fp2_make(c0, c1);
}

// Device call boundary of the Fp2 products (fp.hpp "call-granularity policy"):
//   fp2_mul: ONE call running the lazy-reduction body (five interleaved MAD chains).  The AMDGPU calling
//            convention passes only 32 VGPR arguments in registers, so a0, a1 go as the 28 register arguments and
//            b0, b1 through a per-lane LDS slot (word-major: lane t, word w at bls_fp2_arg[w * 128 + t],
//            conflict-free; every kernel that reaches it has <= 128 lanes per workgroup);
//   fp2_sqr: ONE register-ABI call computing its two products interleaved.
// tools/microbench/fp2_rate.hip (profiles/r02_fp2_rate.json): 1.85e10 Fp2 products/s per chip at one wave per
// SIMD with this call vs 1.39e10 for three fp_mul_r calls.
#if defined(__HIP_DEVICE_COMPILE__) && !BLS_INLINE_PRODUCTS && !BLS_FP2_CLASSIC
#define BLS_FP2_LDS_LANES 128
#if BLSGPU_DEBUG
#include <assert.h>
#endif
__shared__ uint32_t bls_fp2_arg[2 * BLS_NL * BLS_FP2_LDS_LANES];
// The 28-dword result comes back in VGPRs as a 32-wide vector: clang's AMDGPU ABI returns an aggregate of more than
// 16 dwords indirectly (through a scratch sret slot: 7 dwordx4 stores + 7 loads per call), a vector type directly.
typedef uint32_t fp2_ret __attribute__((ext_vector_type(32)));
__device__ __noinline__ fp2_ret fp2_mul_r(BLS_PARAMS14(a), BLS_PARAMS14(c)) {
  const fp x0 = BLS_INIT14(a), x1 = BLS_INIT14(c);
  const uint32_t t = threadIdx.x;
  fp y0, y1;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) {
    y0.l[i] = bls_fp2_arg[i * BLS_FP2_LDS_LANES + t];
    y1.l[i] = bls_fp2_arg[(BLS_NL + i) * BLS_FP2_LDS_LANES + t];
  }
  const fp2 r = fp2_mul_body_sel(x0, x1, y0, y1);
  fp2_ret o;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) {
    o[i] = r.c0.l[i];
    o[BLS_NL + i] = r.c1.l[i];
  }
  return o;
}
__device__ __noinline__ fp2_ret fp2_sqr_r(BLS_PARAMS14(a), BLS_PARAMS14(c)) {
  const fp2 r = fp2_sqr_body(fp2_make(BLS_INIT14(a), BLS_INIT14(c)));
  fp2_ret o;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) {
    o[i] = r.c0.l[i];
    o[BLS_NL + i] = r.c1.l[i];
  }
  return o;
}
__device__ __forceinline__ fp2 fp2_from_ret(const fp2_ret& o) {
  fp2 r;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) {
    r.c0.l[i] = o[i];
    r.c1.l[i] = o[BLS_NL + i];
  }
  return r;
}
__device__ __forceinline__ fp2 fp2_mul(const fp2& a, const fp2& b) {
  const uint32_t t = threadIdx.x;
#if BLSGPU_DEBUG
  // the slot is indexed by threadIdx.x alone: one-dimensional workgroups of <= 128 lanes only
  assert(blockDim.x <= BLS_FP2_LDS_LANES && blockDim.y == 1 && blockDim.z == 1);
#endif
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) {
    bls_fp2_arg[i * BLS_FP2_LDS_LANES + t] = b.c0.l[i];
    bls_fp2_arg[(BLS_NL + i) * BLS_FP2_LDS_LANES + t] = b.c1.l[i];
  }
  return fp2_from_ret(fp2_mul_r(BLS_ARGS14(a.c0), BLS_ARGS14(a.c1)));
}
__device__ __forceinline__ fp2 fp2_sqr(const fp2& a) { return fp2_from_ret(fp2_sqr_r(BLS_ARGS14(a.c0), BLS_ARGS14(a.c1))); }
// a * s (s in Fp, through the LDS slot): two interleaved products in one call
__device__ __noinline__ fp2_ret fp2_mul_fp_r(BLS_PARAMS14(a), BLS_PARAMS14(c)) {
  const fp x0 = BLS_INIT14(a), x1 = BLS_INIT14(c);
  const uint32_t t = threadIdx.x;
  fp y;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) y.l[i] = bls_fp2_arg[i * BLS_FP2_LDS_LANES + t];
  const fp r0 = fp_mul_body(x0, y), r1 = fp_mul_body(x1, y);
  fp2_ret o;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) {
    o[i] = r0.l[i];
    o[BLS_NL + i] = r1.l[i];
  }
  return o;
}
__device__ __forceinline__ fp2 fp2_mul_fp(const fp2& a, const fp& s) {
  const uint32_t t = threadIdx.x;
#if BLSGPU_DEBUG
  assert(blockDim.x <= BLS_FP2_LDS_LANES && blockDim.y == 1 && blockDim.z == 1);
#endif
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) bls_fp2_arg[i * BLS_FP2_LDS_LANES + t] = s.l[i];
  return fp2_from_ret(fp2_mul_fp_r(BLS_ARGS14(a.c0), BLS_ARGS14(a.c1)));
}
#elif BLS_FP2_CLASSIC
// A/B reference (BLSGPU_DEFINES=BLS_FP2_CLASSIC=1): three / two separate product calls, eager reduction
BLS_FN fp2 fp2_mul_fp(const fp2& a, const fp& s) { return fp2_make(fp_mul(a.c0, s), fp_mul(a.c1, s)); }
BLS_FN fp2 fp2_mul(const fp2& a, const fp2& b) {
  fp t0 = fp_mul(a.c0, b.c0);
  fp t1 = fp_mul(a.c1, b.c1);
  fp t2 = fp_mul(fp_add_nr(a.c0, a.c1), fp_add_nr(b.c0, b.c1));
  return fp2_make(fp_sub(t0, t1), fp_sub(fp_sub(t2, t0), t1));
}
BLS_FN fp2 fp2_sqr(const fp2& a) {
  fp c0 = fp_mul(fp_add_nr(a.c0, a.c1), fp_sub_k8(a.c0, a.c1));
  fp c1 = fp_mul(fp_add_nr(a.c0, a.c0), a.c1);
  return fp2_make(c0, c1);
}
#else
BLS_FN fp2 fp2_mul_fp(const fp2& a, const fp& s) { return fp2_make(fp_mul(a.c0, s), fp_mul(a.c1, s)); }
BLS_FN fp2 fp2_mul(const fp2& a, const fp2& b) {
  BLS_COUNT5(bls_count_half);  // 3 half-products + 2 reductions, each half a Montgomery multiplication
  return fp2_mul_body_sel(a.c0, a.c1, b.c0, b.c1);
}
BLS_FN fp2 fp2_sqr(const fp2& a) {
  BLS_COUNT(bls_count_mul);
  BLS_COUNT(bls_count_mul);
  return fp2_sqr_body(a);
}
#endif


// (a0 + a1 u)(1 + u) = (a0 - a1) + (a0 + a1) u
BLS_FN fp2 fp2_mul_xi(const fp2& a) { return fp2_make(fp_sub(a.c0, a.c1), fp_add(a.c0, a.c1)); }

BLS_FN fp2 fp2_mul3(const fp2& a) { return fp2_make(fp_mul3(a.c0), fp_mul3(a.c1)); }

BLS_FN bool fp2_is_zero(const fp2& a) { return fp_is_zero(a.c0) && fp_is_zero(a.c1); }
BLS_FN bool fp2_eq(const fp2& a, const fp2& b) { return fp_eq(a.c0, b.c0) && fp_eq(a.c1, b.c1); }
BLS_HD fp2 fp2_select(bool c, const fp2& a, const fp2& b) {
  return fp2_make(fp_select(c, a.c0, b.c0), fp_select(c, a.c1, b.c1));
}
BLS_FN fp fp2_norm(const fp2& a) {  // a0^2 + a1^2
  return fp_add(fp_sqr(a.c0), fp_sqr(a.c1));
}
BLS_FN fp2 fp2_inv(const fp2& a) {
  fp ni = fp_inv(fp2_norm(a));
  return fp2_make(fp_mul(a.c0, ni), fp_neg(fp_mul(a.c1, ni)));
}

// Square root in Fp2 via the norm (p = 3 mod 4): two Fp exponentiations by (p-3)/4.
// Returns false if `a` is not a square.  Any root may be returned (callers fix the sign).
BLS_HDNI bool fp2_sqrt(const fp2& a, fp2& out) {
  fp n = fp2_norm(a);
  fp e1 = fp_pow_p34(n);
  fp s = fp_mul(n, e1);  // candidate sqrt(n)
  bool ok = fp_eq(fp_sqr(s), n);
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
  out = r;
  bool check = fp2_eq(fp2_sqr(r), a);
  return ok && check;
}

// sgn0 (RFC 9380 4.1) of a canonical plain value pair
BLS_HD uint32_t fp2_sgn0_plain(const fp& c0, const fp& c1) {
  uint32_t s0 = c0.l[0] & 1u;
  uint32_t z0 = 1;
  for (int i = 0; i < BLS_NL; i++) z0 &= (c0.l[i] == 0);
  uint32_t s1 = c1.l[0] & 1u;
  return s0 | (z0 & s1);
}

// ---------------------------------------------------------------------------------------------- Fp6
BLS_HD fp6 fp6_make(const fp2& a, const fp2& b, const fp2& c) {
  fp6 r;
  r.c0 = a;
  r.c1 = b;
  r.c2 = c;
  return r;
}
BLS_HD fp6 fp6_zero() { return fp6_make(fp2_zero(), fp2_zero(), fp2_zero()); }
BLS_HD fp6 fp6_one() { return fp6_make(fp2_one(), fp2_zero(), fp2_zero()); }
BLS_FN fp6 fp6_add(const fp6& a, const fp6& b) { return fp6_make(fp2_add(a.c0, b.c0), fp2_add(a.c1, b.c1), fp2_add(a.c2, b.c2)); }
BLS_FN fp6 fp6_sub(const fp6& a, const fp6& b) { return fp6_make(fp2_sub(a.c0, b.c0), fp2_sub(a.c1, b.c1), fp2_sub(a.c2, b.c2)); }
BLS_FN fp6 fp6_neg(const fp6& a) { return fp6_make(fp2_neg(a.c0), fp2_neg(a.c1), fp2_neg(a.c2)); }
BLS_FN fp6 fp6_mul_v(const fp6& a) { return fp6_make(fp2_mul_xi(a.c2), a.c0, a.c1); }

// Karatsuba over Fp2: six Fp2 products.  The operand sums go to fp2_mul un-normalized (fp2_add_nr): a, b are
// normalized with values <= 4p, so the sums have limbs < 2^29 and values <= 8p -- fp2_mul's input contract.  With
// BLS_LAZY_TOWER each output Fp component is ONE lazily reduced linear combination of product components (fp_lc):
//   c0 = t0 + xi (X - t1 - t2),  c1 = Y - t0 - t1 + xi t2,  c2 = Z - t0 - t2 + t1   (xi (x0 + x1 u) = (x0 - x1) + (x0 + x1) u)
#ifndef BLS_LAZY_TOWER
#define BLS_LAZY_TOWER 1
#endif
#ifndef BLS_LAZY_FP6
#define BLS_LAZY_FP6 BLS_LAZY_TOWER
#endif
#ifndef BLS_LAZY_SQR
#define BLS_LAZY_SQR BLS_LAZY_TOWER
#endif
#ifndef BLS_LAZY_014
#define BLS_LAZY_014 BLS_LAZY_TOWER
#endif
#if BLS_LAZY_FP6
BLS_FN fp6 fp6_mul(const fp6& a, const fp6& b) {
  const fp2 t0 = fp2_mul(a.c0, b.c0);
  const fp2 t1 = fp2_mul(a.c1, b.c1);
  const fp2 t2 = fp2_mul(a.c2, b.c2);
  fp6 r;
  {
    const fp2 X = fp2_mul(fp2_add_nr(a.c1, a.c2), fp2_add_nr(b.c1, b.c2));
    r.c0.c0 = fp_lc(T<1>(t0.c0), T<1>(X.c0), T<-1>(t1.c0), T<-1>(t2.c0), T<-1>(X.c1), T<1>(t1.c1), T<1>(t2.c1));
    r.c0.c1 = fp_lc(T<1>(t0.c1), T<1>(X.c0), T<-1>(t1.c0), T<-1>(t2.c0), T<1>(X.c1), T<-1>(t1.c1), T<-1>(t2.c1));
  }
  {
    const fp2 Y = fp2_mul(fp2_add_nr(a.c0, a.c1), fp2_add_nr(b.c0, b.c1));
    r.c1.c0 = fp_lc(T<1>(Y.c0), T<-1>(t0.c0), T<-1>(t1.c0), T<1>(t2.c0), T<-1>(t2.c1));
    r.c1.c1 = fp_lc(T<1>(Y.c1), T<-1>(t0.c1), T<-1>(t1.c1), T<1>(t2.c0), T<1>(t2.c1));
  }
  {
    const fp2 Z = fp2_mul(fp2_add_nr(a.c0, a.c2), fp2_add_nr(b.c0, b.c2));
    r.c2.c0 = fp_lc(T<1>(Z.c0), T<-1>(t0.c0), T<-1>(t2.c0), T<1>(t1.c0));
    r.c2.c1 = fp_lc(T<1>(Z.c1), T<-1>(t0.c1), T<-1>(t2.c1), T<1>(t1.c1));
  }
  return r;
}
#else
BLS_FN fp6 fp6_mul(const fp6& a, const fp6& b) {
  fp2 t0 = fp2_mul(a.c0, b.c0);
  fp2 t1 = fp2_mul(a.c1, b.c1);
  fp2 t2 = fp2_mul(a.c2, b.c2);
  fp2 c0 = fp2_add(t0, fp2_mul_xi(fp2_sub(fp2_mul(fp2_add_nr(a.c1, a.c2), fp2_add_nr(b.c1, b.c2)), fp2_add(t1, t2))));
  fp2 c1 = fp2_add(fp2_sub(fp2_mul(fp2_add_nr(a.c0, a.c1), fp2_add_nr(b.c0, b.c1)), fp2_add(t0, t1)), fp2_mul_xi(t2));
  fp2 c2 = fp2_add(fp2_sub(fp2_mul(fp2_add_nr(a.c0, a.c2), fp2_add_nr(b.c0, b.c2)), fp2_add(t0, t2)), t1);
  return fp6_make(c0, c1, c2);
}

#endif

// (x0 + x1 v + x2 v^2)(l0 + l1 v): t0 = x0 l0, t1 = x1 l1, c0 = t0 + xi (x2 l1), c1 = (x0 + x1)(l0 + l1) - t0 - t1,
// c2 = x2 l0 + t1 -- five Fp2 products (x, l normalized, values <= 4p)
#if BLS_LAZY_FP6
BLS_FN fp6 fp6_mul_by_01(const fp6& x, const fp2& l0, const fp2& l1) {
  const fp2 t0 = fp2_mul(x.c0, l0);
  const fp2 t1 = fp2_mul(x.c1, l1);
  fp6 r;
  {
    const fp2 u = fp2_mul(x.c2, l1);
    r.c0.c0 = fp_lc(T<1>(t0.c0), T<1>(u.c0), T<-1>(u.c1));
    r.c0.c1 = fp_lc(T<1>(t0.c1), T<1>(u.c0), T<1>(u.c1));
  }
  {
    const fp2 v = fp2_mul(fp2_add_nr(x.c0, x.c1), fp2_add_nr(l0, l1));
    r.c1.c0 = fp_lc(T<1>(v.c0), T<-1>(t0.c0), T<-1>(t1.c0));
    r.c1.c1 = fp_lc(T<1>(v.c1), T<-1>(t0.c1), T<-1>(t1.c1));
  }
  {
    const fp2 w = fp2_mul(x.c2, l0);
    r.c2.c0 = fp_lc(T<1>(w.c0), T<1>(t1.c0));
    r.c2.c1 = fp_lc(T<1>(w.c1), T<1>(t1.c1));
  }
  return r;
}
#else
BLS_FN fp6 fp6_mul_by_01(const fp6& x, const fp2& l0, const fp2& l1) {
  fp2 t0 = fp2_mul(x.c0, l0);
  fp2 t1 = fp2_mul(x.c1, l1);
  fp2 c0 = fp2_add(t0, fp2_mul_xi(fp2_mul(x.c2, l1)));
  fp2 c1 = fp2_sub(fp2_sub(fp2_mul(fp2_add_nr(x.c0, x.c1), fp2_add_nr(l0, l1)), t0), t1);  // (see fp6_mul)
  fp2 c2 = fp2_add(fp2_mul(x.c2, l0), t1);
  return fp6_make(c0, c1, c2);
}

#endif

// (x0 + x1 v + x2 v^2) * (l1 v)
BLS_FN fp6 fp6_mul_by_1(const fp6& x, const fp2& l1) {
  return fp6_make(fp2_mul_xi(fp2_mul(x.c2, l1)), fp2_mul(x.c0, l1), fp2_mul(x.c1, l1));
}

BLS_BIG fp6 fp6_inv(const fp6& a) {
  fp2 t0 = fp2_sub(fp2_sqr(a.c0), fp2_mul_xi(fp2_mul(a.c1, a.c2)));
  fp2 t1 = fp2_sub(fp2_mul_xi(fp2_sqr(a.c2)), fp2_mul(a.c0, a.c1));
  fp2 t2 = fp2_sub(fp2_sqr(a.c1), fp2_mul(a.c0, a.c2));
  fp2 d = fp2_add(fp2_mul(a.c0, t0), fp2_mul_xi(fp2_add(fp2_mul(a.c2, t1), fp2_mul(a.c1, t2))));
  fp2 di = fp2_inv(d);
  return fp6_make(fp2_mul(t0, di), fp2_mul(t1, di), fp2_mul(t2, di));
}

// X - A - B component-wise as lazy combinations (terms: products, normalized, values <= 2p)
#define F2_LC3(X, A, B) \
  fp2_make(fp_lc(T<1>((X).c0), T<-1>((A).c0), T<-1>((B).c0)), fp_lc(T<1>((X).c1), T<-1>((A).c1), T<-1>((B).c1)))
// --------------------------------------------------------------------------------------------- Fp12
BLS_HD fp12 fp12_make(const fp6& a, const fp6& b) {
  fp12 r;
  r.c0 = a;
  r.c1 = b;
  return r;
}
BLS_HD fp12 fp12_one() { return fp12_make(fp6_one(), fp6_zero()); }

#if BLS_LAZY_FP6
// Karatsuba over Fp6 (fp6_mul's lazy contract: operand sums normalized, not reduced, values <= 4p);
// c0 = t0 + v t1 = (t0.c0 + xi t1.c2, t0.c1 + t1.c0, t0.c2 + t1.c1), c1 = X - t0 - t1.
BLS_FN fp12 fp12_mul(const fp12& a, const fp12& b) {
  const fp6 t0 = fp6_mul(a.c0, b.c0);
  const fp6 t1 = fp6_mul(a.c1, b.c1);
  fp6 sa, sb;
  sa.c0 = fp2_make(fp_add_norm(a.c0.c0.c0, a.c1.c0.c0), fp_add_norm(a.c0.c0.c1, a.c1.c0.c1));
  sa.c1 = fp2_make(fp_add_norm(a.c0.c1.c0, a.c1.c1.c0), fp_add_norm(a.c0.c1.c1, a.c1.c1.c1));
  sa.c2 = fp2_make(fp_add_norm(a.c0.c2.c0, a.c1.c2.c0), fp_add_norm(a.c0.c2.c1, a.c1.c2.c1));
  sb.c0 = fp2_make(fp_add_norm(b.c0.c0.c0, b.c1.c0.c0), fp_add_norm(b.c0.c0.c1, b.c1.c0.c1));
  sb.c1 = fp2_make(fp_add_norm(b.c0.c1.c0, b.c1.c1.c0), fp_add_norm(b.c0.c1.c1, b.c1.c1.c1));
  sb.c2 = fp2_make(fp_add_norm(b.c0.c2.c0, b.c1.c2.c0), fp_add_norm(b.c0.c2.c1, b.c1.c2.c1));
  const fp6 X = fp6_mul(sa, sb);
  fp12 r;
  r.c0.c0 = fp2_make(fp_lc(T<1>(t0.c0.c0), T<1>(t1.c2.c0), T<-1>(t1.c2.c1)),
                     fp_lc(T<1>(t0.c0.c1), T<1>(t1.c2.c0), T<1>(t1.c2.c1)));
  r.c0.c1 = fp2_make(fp_lc(T<1>(t0.c1.c0), T<1>(t1.c0.c0)), fp_lc(T<1>(t0.c1.c1), T<1>(t1.c0.c1)));
  r.c0.c2 = fp2_make(fp_lc(T<1>(t0.c2.c0), T<1>(t1.c1.c0)), fp_lc(T<1>(t0.c2.c1), T<1>(t1.c1.c1)));
  r.c1.c0 = fp2_make(fp_lc(T<1>(X.c0.c0), T<-1>(t0.c0.c0), T<-1>(t1.c0.c0)),
                     fp_lc(T<1>(X.c0.c1), T<-1>(t0.c0.c1), T<-1>(t1.c0.c1)));
  r.c1.c1 = fp2_make(fp_lc(T<1>(X.c1.c0), T<-1>(t0.c1.c0), T<-1>(t1.c1.c0)),
                     fp_lc(T<1>(X.c1.c1), T<-1>(t0.c1.c1), T<-1>(t1.c1.c1)));
  r.c1.c2 = fp2_make(fp_lc(T<1>(X.c2.c0), T<-1>(t0.c2.c0), T<-1>(t1.c2.c0)),
                     fp_lc(T<1>(X.c2.c1), T<-1>(t0.c2.c1), T<-1>(t1.c2.c1)));
  return r;
}
#else
BLS_FN fp12 fp12_mul(const fp12& a, const fp12& b) {
  fp6 t0 = fp6_mul(a.c0, b.c0);
  fp6 t1 = fp6_mul(a.c1, b.c1);
  fp6 c1 = fp6_sub(fp6_mul(fp6_add(a.c0, a.c1), fp6_add(b.c0, b.c1)), fp6_add(t0, t1));
  fp6 c0 = fp6_add(t0, fp6_mul_v(t1));
  return fp12_make(c0, c1);
}
#endif

// (a0 + a1 w)^2 = (a0^2 + v a1^2) + 2 a0 a1 w ;  complex-method squaring, 2 Fp6 muls
#if BLS_LAZY_SQR
// u = a0 + a1 and w = a0 + v a1 as fp6_mul operands (normalized, values <= 4p: carry pass only, no reduction, except
// w.c0 = a0.c0 + xi a1.c2, a signed combination); c0 = s - t - v t, c1 = 2 t as combinations of the reduced s, t.
BLS_FN fp12 fp12_sqr(const fp12& a) {
  const fp6 t = fp6_mul(a.c0, a.c1);
  fp6 u, w;
  u.c0 = fp2_make(fp_add_norm(a.c0.c0.c0, a.c1.c0.c0), fp_add_norm(a.c0.c0.c1, a.c1.c0.c1));
  u.c1 = fp2_make(fp_add_norm(a.c0.c1.c0, a.c1.c1.c0), fp_add_norm(a.c0.c1.c1, a.c1.c1.c1));
  u.c2 = fp2_make(fp_add_norm(a.c0.c2.c0, a.c1.c2.c0), fp_add_norm(a.c0.c2.c1, a.c1.c2.c1));
  w.c0 = fp2_make(fp_lc(T<1>(a.c0.c0.c0), T<1>(a.c1.c2.c0), T<-1>(a.c1.c2.c1)),
                  fp_lc(T<1>(a.c0.c0.c1), T<1>(a.c1.c2.c0), T<1>(a.c1.c2.c1)));
  w.c1 = fp2_make(fp_add_norm(a.c0.c1.c0, a.c1.c0.c0), fp_add_norm(a.c0.c1.c1, a.c1.c0.c1));
  w.c2 = fp2_make(fp_add_norm(a.c0.c2.c0, a.c1.c1.c0), fp_add_norm(a.c0.c2.c1, a.c1.c1.c1));
  const fp6 s = fp6_mul(u, w);
  fp12 r;
  // v t = (xi t2, t0, t1)
  r.c0.c0.c0 = fp_lc(T<1>(s.c0.c0), T<-1>(t.c0.c0), T<-1>(t.c2.c0), T<1>(t.c2.c1));
  r.c0.c0.c1 = fp_lc(T<1>(s.c0.c1), T<-1>(t.c0.c1), T<-1>(t.c2.c0), T<-1>(t.c2.c1));
  r.c0.c1.c0 = fp_lc(T<1>(s.c1.c0), T<-1>(t.c1.c0), T<-1>(t.c0.c0));
  r.c0.c1.c1 = fp_lc(T<1>(s.c1.c1), T<-1>(t.c1.c1), T<-1>(t.c0.c1));
  r.c0.c2.c0 = fp_lc(T<1>(s.c2.c0), T<-1>(t.c2.c0), T<-1>(t.c1.c0));
  r.c0.c2.c1 = fp_lc(T<1>(s.c2.c1), T<-1>(t.c2.c1), T<-1>(t.c1.c1));
  r.c1.c0 = fp2_make(fp_lc(T<2>(t.c0.c0)), fp_lc(T<2>(t.c0.c1)));
  r.c1.c1 = fp2_make(fp_lc(T<2>(t.c1.c0)), fp_lc(T<2>(t.c1.c1)));
  r.c1.c2 = fp2_make(fp_lc(T<2>(t.c2.c0)), fp_lc(T<2>(t.c2.c1)));
  return r;
}
#else
BLS_FN fp12 fp12_sqr(const fp12& a) {
  fp6 t = fp6_mul(a.c0, a.c1);
  fp6 s = fp6_mul(fp6_add(a.c0, a.c1), fp6_add(a.c0, fp6_mul_v(a.c1)));
  fp6 c0 = fp6_sub(fp6_sub(s, t), fp6_mul_v(t));
  fp6 c1 = fp6_add(t, t);
  return fp12_make(c0, c1);
}
#endif

BLS_HD fp12 fp12_conj(const fp12& a) { return fp12_make(a.c0, fp6_neg(a.c1)); }

BLS_BIG fp12 fp12_inv(const fp12& a) {
  fp6 t = fp6_sub(fp6_mul(a.c0, a.c0), fp6_mul_v(fp6_mul(a.c1, a.c1)));
  fp6 ti = fp6_inv(t);
  return fp12_make(fp6_mul(a.c0, ti), fp6_neg(fp6_mul(a.c1, ti)));
}

// f * line, line = l0 + l1 v + l4 v w   (positions c0.c0, c0.c1, c1.c1) -- 13 Fp2 multiplications
#if BLS_LAZY_014
// A0 = f0 (l0 + l1 v) (reduced), A1 = f1 (l4 v) = (xi Q1, Q2, Q3) with Qk = f1.c(k-1 mod 3) l4 kept as raw products,
// S = (f0 + f1)(l0 + (l1 + l4) v); c0 = A0 + v A1 = (A0.c0 + xi Q3, A0.c1 + xi Q1, A0.c2 + Q2), c1 = S - A0 - A1 with
// S's five products folded straight into c1's combinations.  f, l: normalized, values <= 2p.
BLS_FN fp12 fp12_mul_by_014(const fp12& f, const fp2& l0, const fp2& l1, const fp2& l4) {
  fp6 b;  // f0 + f1 (values <= 4p, normalized)
  b.c0 = fp2_make(fp_add_norm(f.c0.c0.c0, f.c1.c0.c0), fp_add_norm(f.c0.c0.c1, f.c1.c0.c1));
  b.c1 = fp2_make(fp_add_norm(f.c0.c1.c0, f.c1.c1.c0), fp_add_norm(f.c0.c1.c1, f.c1.c1.c1));
  b.c2 = fp2_make(fp_add_norm(f.c0.c2.c0, f.c1.c2.c0), fp_add_norm(f.c0.c2.c1, f.c1.c2.c1));
  const fp2 Q1 = fp2_mul(f.c1.c2, l4), Q2 = fp2_mul(f.c1.c0, l4), Q3 = fp2_mul(f.c1.c1, l4);
  const fp6 A0 = fp6_mul_by_01(f.c0, l0, l1);
  fp12 r;
  r.c0.c0 = fp2_make(fp_lc(T<1>(A0.c0.c0), T<1>(Q3.c0), T<-1>(Q3.c1)), fp_lc(T<1>(A0.c0.c1), T<1>(Q3.c0), T<1>(Q3.c1)));
  r.c0.c1 = fp2_make(fp_lc(T<1>(A0.c1.c0), T<1>(Q1.c0), T<-1>(Q1.c1)), fp_lc(T<1>(A0.c1.c1), T<1>(Q1.c0), T<1>(Q1.c1)));
  r.c0.c2 = fp2_make(fp_lc(T<1>(A0.c2.c0), T<1>(Q2.c0)), fp_lc(T<1>(A0.c2.c1), T<1>(Q2.c1)));
  // S = b (l0 + m v), m = l1 + l4: R1 = b0 l0, R2 = b1 m, R3 = b2 m, R4 = (b0 + b1)(l0 + m), R5 = b2 l0;
  // S = (R1 + xi R3, R4 - R1 - R2, R5 + R2)
  const fp2 m = fp2_make(fp_add_norm(l1.c0, l4.c0), fp_add_norm(l1.c1, l4.c1));
  const fp2 R1 = fp2_mul(b.c0, l0), R2 = fp2_mul(b.c1, m);
  {
    const fp2 R4 = fp2_mul(fp2_add_nr(b.c0, b.c1), fp2_add_nr(l0, m));
    r.c1.c1 = fp2_make(fp_lc(T<1>(R4.c0), T<-1>(R1.c0), T<-1>(R2.c0), T<-1>(A0.c1.c0), T<-1>(Q2.c0)),
                       fp_lc(T<1>(R4.c1), T<-1>(R1.c1), T<-1>(R2.c1), T<-1>(A0.c1.c1), T<-1>(Q2.c1)));
  }
  {
    const fp2 R3 = fp2_mul(b.c2, m);
    r.c1.c0 = fp2_make(fp_lc(T<1>(R1.c0), T<1>(R3.c0), T<-1>(R3.c1), T<-1>(A0.c0.c0), T<-1>(Q1.c0), T<1>(Q1.c1)),
                       fp_lc(T<1>(R1.c1), T<1>(R3.c0), T<1>(R3.c1), T<-1>(A0.c0.c1), T<-1>(Q1.c0), T<-1>(Q1.c1)));
  }
  {
    const fp2 R5 = fp2_mul(b.c2, l0);
    r.c1.c2 = fp2_make(fp_lc(T<1>(R5.c0), T<1>(R2.c0), T<-1>(A0.c2.c0), T<-1>(Q3.c0)),
                       fp_lc(T<1>(R5.c1), T<1>(R2.c1), T<-1>(A0.c2.c1), T<-1>(Q3.c1)));
  }
  return r;
}
#else
BLS_FN fp12 fp12_mul_by_014(const fp12& f, const fp2& l0, const fp2& l1, const fp2& l4) {
  fp6 a0 = fp6_mul_by_01(f.c0, l0, l1);
  fp6 a1 = fp6_mul_by_1(f.c1, l4);
  fp6 s = fp6_mul_by_01(fp6_add(f.c0, f.c1), l0, fp2_add(l1, l4));
  fp6 c1 = fp6_sub(fp6_sub(s, a0), a1);
  fp6 c0 = fp6_add(a0, fp6_mul_v(a1));
  return fp12_make(c0, c1);
}
#endif

// Two lines multiplied together first (the Miller accumulation's chunks of two pairings): (a0 + a1 v + a4 v w)
// (b0 + b1 v + b4 v w) = (a0 b0 + xi a4 b4) + (a0 b1 + a1 b0) v + a1 b1 v^2 + (a0 b4 + a4 b0) v w + (a1 b4 + a4 b1) v^2 w
// (w^2 = v, v^3 = xi): six Fp2 products (three squares of the pairs by Karatsuba), c1.c0 = 0.  Then f times that
// element (fp12_mul_by_line2: 17 products) -- 23 in all against 26 for two sparse products.  Inputs normalized,
// values <= 2p; outputs lazily reduced (fp_lc).
BLS_FN fp12 line_pair(const fp2& a0, const fp2& a1, const fp2& a4, const fp2& b0, const fp2& b1, const fp2& b4) {
  const fp2 P00 = fp2_mul(a0, b0), P11 = fp2_mul(a1, b1), P44 = fp2_mul(a4, b4);
  fp12 m;
  m.c0.c0 = fp2_make(fp_lc(T<1>(P00.c0), T<1>(P44.c0), T<-1>(P44.c1)), fp_lc(T<1>(P00.c1), T<1>(P44.c0), T<1>(P44.c1)));
  m.c0.c2 = P11;
  m.c1.c0 = fp2_zero();
  {
    const fp2 X = fp2_mul(fp2_add_nr(a0, a1), fp2_add_nr(b0, b1));
    m.c0.c1 = F2_LC3(X, P00, P11);
  }
  {
    const fp2 X = fp2_mul(fp2_add_nr(a0, a4), fp2_add_nr(b0, b4));
    m.c1.c1 = F2_LC3(X, P00, P44);
  }
  {
    const fp2 X = fp2_mul(fp2_add_nr(a1, a4), fp2_add_nr(b1, b4));
    m.c1.c2 = F2_LC3(X, P11, P44);
  }
  return m;
}

// f * m with m.c1.c0 = 0 (a line_pair product): Karatsuba over Fp6, t1 = f1 m1 with m1 = (0, b1, b2) in five
// products: c0 = xi (X - t1 - t2), c1 = (a0 + a1) b1 - t1 + xi t2, c2 = (a0 + a2) b2 - t2 + t1, X = (a1 + a2)(b1 + b2)
BLS_FN fp6 fp6_mul_by_12(const fp6& a, const fp2& b1, const fp2& b2) {
  const fp2 t1 = fp2_mul(a.c1, b1), t2 = fp2_mul(a.c2, b2);
  fp6 r;
  {
    const fp2 X = fp2_mul(fp2_add_nr(a.c1, a.c2), fp2_add_nr(b1, b2));  // X - t1 - t2 = a1 b2 + a2 b1
    r.c0.c0 = fp_lc(T<1>(X.c0), T<-1>(t1.c0), T<-1>(t2.c0), T<-1>(X.c1), T<1>(t1.c1), T<1>(t2.c1));
    r.c0.c1 = fp_lc(T<1>(X.c0), T<-1>(t1.c0), T<-1>(t2.c0), T<1>(X.c1), T<-1>(t1.c1), T<-1>(t2.c1));
  }
  {
    const fp2 Y = fp2_mul(fp2_add_nr(a.c0, a.c1), b1);
    r.c1.c0 = fp_lc(T<1>(Y.c0), T<-1>(t1.c0), T<1>(t2.c0), T<-1>(t2.c1));
    r.c1.c1 = fp_lc(T<1>(Y.c1), T<-1>(t1.c1), T<1>(t2.c0), T<1>(t2.c1));
  }
  {
    const fp2 Z = fp2_mul(fp2_add_nr(a.c0, a.c2), b2);
    r.c2.c0 = fp_lc(T<1>(Z.c0), T<-1>(t2.c0), T<1>(t1.c0));
    r.c2.c1 = fp_lc(T<1>(Z.c1), T<-1>(t2.c1), T<1>(t1.c1));
  }
  return r;
}
BLS_FN fp12 fp12_mul_by_line2(const fp12& f, const fp12& m) {
  const fp6 t0 = fp6_mul(f.c0, m.c0);
  const fp6 t1 = fp6_mul_by_12(f.c1, m.c1.c1, m.c1.c2);
  fp6 sa, sb;  // f0 + f1, m0 + m1 (normalized, values <= 4p: fp6_mul's operand contract)
  sa.c0 = fp2_make(fp_add_norm(f.c0.c0.c0, f.c1.c0.c0), fp_add_norm(f.c0.c0.c1, f.c1.c0.c1));
  sa.c1 = fp2_make(fp_add_norm(f.c0.c1.c0, f.c1.c1.c0), fp_add_norm(f.c0.c1.c1, f.c1.c1.c1));
  sa.c2 = fp2_make(fp_add_norm(f.c0.c2.c0, f.c1.c2.c0), fp_add_norm(f.c0.c2.c1, f.c1.c2.c1));
  sb.c0 = m.c0.c0;
  sb.c1 = fp2_make(fp_add_norm(m.c0.c1.c0, m.c1.c1.c0), fp_add_norm(m.c0.c1.c1, m.c1.c1.c1));
  sb.c2 = fp2_make(fp_add_norm(m.c0.c2.c0, m.c1.c2.c0), fp_add_norm(m.c0.c2.c1, m.c1.c2.c1));
  const fp6 X = fp6_mul(sa, sb);
  fp12 r;  // c0 = t0 + v t1 = (t0.c0 + xi t1.c2, t0.c1 + t1.c0, t0.c2 + t1.c1), c1 = X - t0 - t1
  r.c0.c0 = fp2_make(fp_lc(T<1>(t0.c0.c0), T<1>(t1.c2.c0), T<-1>(t1.c2.c1)),
                     fp_lc(T<1>(t0.c0.c1), T<1>(t1.c2.c0), T<1>(t1.c2.c1)));
  r.c0.c1 = fp2_make(fp_lc(T<1>(t0.c1.c0), T<1>(t1.c0.c0)), fp_lc(T<1>(t0.c1.c1), T<1>(t1.c0.c1)));
  r.c0.c2 = fp2_make(fp_lc(T<1>(t0.c2.c0), T<1>(t1.c1.c0)), fp_lc(T<1>(t0.c2.c1), T<1>(t1.c1.c1)));
  r.c1.c0 = fp2_make(fp_lc(T<1>(X.c0.c0), T<-1>(t0.c0.c0), T<-1>(t1.c0.c0)),
                     fp_lc(T<1>(X.c0.c1), T<-1>(t0.c0.c1), T<-1>(t1.c0.c1)));
  r.c1.c1 = fp2_make(fp_lc(T<1>(X.c1.c0), T<-1>(t0.c1.c0), T<-1>(t1.c1.c0)),
                     fp_lc(T<1>(X.c1.c1), T<-1>(t0.c1.c1), T<-1>(t1.c1.c1)));
  r.c1.c2 = fp2_make(fp_lc(T<1>(X.c2.c0), T<-1>(t0.c2.c0), T<-1>(t1.c2.c0)),
                     fp_lc(T<1>(X.c2.c1), T<-1>(t0.c2.c1), T<-1>(t1.c2.c1)));
  return r;
}

// Squaring in the cyclotomic subgroup (Granger-Scott, eprint 2009/565 section 3.2): f^(p^6+1) = 1 lets
// f^2 be computed from three Fp4 squarings -- 9 Fp2 squarings (18 Fp products) instead of 36.
// Only valid after the easy part of the final exponentiation.
BLS_INL void fp4_sqr(const fp2& a, const fp2& b, fp2& c0, fp2& c1) {
  fp2 t0 = fp2_sqr(a);
  fp2 t1 = fp2_sqr(b);
  c0 = fp2_add(fp2_mul_xi(t1), t0);
  c1 = fp2_sub(fp2_sub(fp2_sqr(fp2_add(a, b)), t0), t1);
}
BLS_INL fp2 cyc_fix_sub(const fp2& t, const fp2& z) {  // 2 (t - z) + t = 3t - 2z
  fp2 d = fp2_sub(t, z);
  return fp2_add(fp2_dbl(d), t);
}
BLS_INL fp2 cyc_fix_add(const fp2& t, const fp2& z) {  // 2 (t + z) + t = 3t + 2z
  fp2 d = fp2_add(t, z);
  return fp2_add(fp2_dbl(d), t);
}
BLS_INL fp12 fp12_cyclotomic_sqr(const fp12& f) {
  fp2 t0, t1, t2, t3, u0, u1;
  fp4_sqr(f.c0.c0, f.c1.c1, t0, t1);
  fp12 r;
  r.c0.c0 = cyc_fix_sub(t0, f.c0.c0);
  r.c1.c1 = cyc_fix_add(t1, f.c1.c1);
  fp4_sqr(f.c1.c0, f.c0.c2, u0, u1);
  fp4_sqr(f.c0.c1, f.c1.c2, t2, t3);
  r.c0.c1 = cyc_fix_sub(u0, f.c0.c1);
  r.c1.c2 = cyc_fix_add(u1, f.c1.c2);
  r.c1.c0 = cyc_fix_add(fp2_mul_xi(t3), f.c1.c0);
  r.c0.c2 = cyc_fix_sub(t2, f.c0.c2);
  return r;
}

// Frobenius x -> x^(p^k) for k = 1, 2, 3
BLS_FN fp12 fp12_frob1(const fp12& a) {
  fp12 r;
  r.c0.c0 = fp2_conj(a.c0.c0);
  r.c1.c0 = fp2_mul(fp2_conj(a.c1.c0), FROB1_1);
  r.c0.c1 = fp2_mul(fp2_conj(a.c0.c1), FROB1_2);
  r.c1.c1 = fp2_mul(fp2_conj(a.c1.c1), FROB1_3);
  r.c0.c2 = fp2_mul(fp2_conj(a.c0.c2), FROB1_4);
  r.c1.c2 = fp2_mul(fp2_conj(a.c1.c2), FROB1_5);
  return r;
}
BLS_FN fp12 fp12_frob2(const fp12& a) {
  fp12 r;
  r.c0.c0 = a.c0.c0;
  r.c1.c0 = fp2_mul(a.c1.c0, FROB2_1);
  r.c0.c1 = fp2_mul(a.c0.c1, FROB2_2);
  r.c1.c1 = fp2_mul(a.c1.c1, FROB2_3);
  r.c0.c2 = fp2_mul(a.c0.c2, FROB2_4);
  r.c1.c2 = fp2_mul(a.c1.c2, FROB2_5);
  return r;
}

BLS_BIG bool fp12_is_one(const fp12& a) {
  bool r = fp2_eq(a.c0.c0, fp2_one());
  r = r && fp2_is_zero(a.c0.c1) && fp2_is_zero(a.c0.c2);
  r = r && fp2_is_zero(a.c1.c0) && fp2_is_zero(a.c1.c1) && fp2_is_zero(a.c1.c2);
  return r;
}

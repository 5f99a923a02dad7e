// Base field Fp of BLS12-381 for gfx950 (CDNA4) VALU.
//
// Representation: 14 limbs x 28 bits, Montgomery form with R = 2^392.  The limb width is chosen for
// gfx950's integer pipes (measured, profiles/r01_valu_rates.json): v_mad_u64_u32 (32x32+64 -> 64)
// issues at half rate, and so do the carry-flag adds (v_add_co/v_addc_co) -- but a 28-bit limb product
// is < 2^56, so every Montgomery column (up to 28 products) is summed by plain v_mad_u64_u32 with NO
// carry flags at all.  One Montgomery multiplication = 392 v_mad_u64_u32 (14^2 a*b + 14^2 m*p),
// one squaring = 301.
//
// Value invariant for every stored element: 0 <= value <= 2p, limbs normalized (< 2^28, top limb holds
// the rest).  fp_mul/fp_sqr outputs are < p + 2^-6 p.  Operands of fp_mul may be un-normalized sums
// (`fp_add_nr`) of up to 4 invariant values (limbs < 2^30); fp_sqr accepts one level (limbs < 2^29).
//
// Reference semantics replaced: blst's vec384/mul_mont_384 family inside @chainsafe/blst@0.2.4
// (reference yarn.lock:445-451) -- restated from the field definition, not translated.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
// Device-only under hipcc: the host pass of a kernel TU must not compile (and fully inline) the
// arithmetic for x86.  The host build of the same headers (tests/native/emu.cpp, g++) takes the #else.
#define BLS_HD __device__ __forceinline__
// Call-granularity policy.  AMDGPU passes aggregate arguments larger than 16 dwords through scratch and
// a caller cannot keep its live values in registers a callee may clobber, so a device function whose
// arguments are Fp/Fp2/Fp12 values costs a scratch round trip per call.  Therefore:
//   * the two Montgomery products are register-ABI calls (fp_mul_r / fp_sqr_r below: operands as 28 / 14
//     scalar VGPR arguments, the 14-dword result returned in VGPRs -- no scratch, ~42 v_mov per call),
//     which keeps every call site ~50 instructions and the compile time of the whole pipeline small;
//   * everything between a product and a coarse loop (Fp/Fp2/Fp6/Fp12 algebra, point formulas, Miller
//     steps) is inlined, so it runs on register-resident values;
//   * only coarse operations that loop internally (exponentiations, scalar multiplications, the Miller
//     loop, the final exponentiation, decoders) are real device functions (BLS_BIG / BLS_HDNI), where the
//     argument round trip is negligible next to their work.
#define BLS_INL __device__ __forceinline__
#if BLS_INLINE_BIG
#define BLS_BIG __device__ __forceinline__
#else
#define BLS_BIG __device__ __noinline__
#endif
#define BLS_HDNI BLS_BIG
#define BLS_FN BLS_INL
#else
#define BLS_HD static inline
#define BLS_HDNI static
#define BLS_FN static inline
#define BLS_INL static inline
#define BLS_BIG static
#endif
#define BLS_CONST static constexpr

#define BLS_NL 14
#define BLS_LB 28
#define BLS_MASK 0x0FFFFFFFu

struct fp {
  uint32_t l[BLS_NL];
};
struct fp2 {
  fp c0, c1;
};

#include "bls_constants.hpp"

// Host-only instrumentation (tests/native/emu.cpp with -DBLS_COUNT_OPS): counts Montgomery
// multiplications / squarings of the device algorithm to give the roofline its algorithmic work.
#if defined(BLS_COUNT_OPS) && !defined(__HIP_DEVICE_COMPILE__)
extern unsigned long long bls_count_mul, bls_count_sqr, bls_count_half;
#define BLS_COUNT(x) (x++)
#define BLS_COUNT5(x) (x += 5)
#else
#define BLS_COUNT(x) ((void)0)
#define BLS_COUNT5(x) ((void)0)
#endif

// ------------------------------------------------------------------------------------------------
// Montgomery multiplication: finely integrated product scanning (column-wise a*b and m*p).
// ------------------------------------------------------------------------------------------------
BLS_INL fp fp_mul_body(const fp& a, const fp& b) {
  fp r;
  uint32_t m[BLS_NL];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < BLS_NL; k++) {
#pragma unroll
    for (int i = 0; i <= k; i++) acc += (uint64_t)a.l[i] * b.l[k - i];
#pragma unroll
    for (int i = 0; i < k; i++) acc += (uint64_t)m[i] * FP_P.l[k - i];
    uint32_t mk = ((uint32_t)acc * BLS_N0INV) & BLS_MASK;
    m[k] = mk;
    acc += (uint64_t)mk * FP_P.l[0];
    acc >>= BLS_LB;
  }
#pragma unroll
  for (int k = BLS_NL; k < 2 * BLS_NL - 1; k++) {
#pragma unroll
    for (int i = k - BLS_NL + 1; i < BLS_NL; i++) {
      acc += (uint64_t)a.l[i] * b.l[k - i];
      acc += (uint64_t)m[i] * FP_P.l[k - i];
    }
    r.l[k - BLS_NL] = (uint32_t)acc & BLS_MASK;
    acc >>= BLS_LB;
  }
  r.l[BLS_NL - 1] = (uint32_t)acc;
  return r;
}

BLS_INL fp fp_sqr_body(const fp& a) {
  fp r;
  uint32_t m[BLS_NL];
  uint32_t a2[BLS_NL];
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) a2[i] = a.l[i] << 1;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < BLS_NL; k++) {
#pragma unroll
    for (int i = 0; 2 * i < k; i++) acc += (uint64_t)a2[i] * a.l[k - i];
    if ((k & 1) == 0) acc += (uint64_t)a.l[k >> 1] * a.l[k >> 1];
#pragma unroll
    for (int i = 0; i < k; i++) acc += (uint64_t)m[i] * FP_P.l[k - i];
    uint32_t mk = ((uint32_t)acc * BLS_N0INV) & BLS_MASK;
    m[k] = mk;
    acc += (uint64_t)mk * FP_P.l[0];
    acc >>= BLS_LB;
  }
#pragma unroll
  for (int k = BLS_NL; k < 2 * BLS_NL - 1; k++) {
#pragma unroll
    for (int i = k - BLS_NL + 1; 2 * i < k; i++) acc += (uint64_t)a2[i] * a.l[k - i];
    if ((k & 1) == 0) acc += (uint64_t)a.l[k >> 1] * a.l[k >> 1];
#pragma unroll
    for (int i = k - BLS_NL + 1; i < BLS_NL; i++) acc += (uint64_t)m[i] * FP_P.l[k - i];
    r.l[k - BLS_NL] = (uint32_t)acc & BLS_MASK;
    acc >>= BLS_LB;
  }
  r.l[BLS_NL - 1] = (uint32_t)acc;
  return r;
}

// Register-ABI product boundary (see the call-granularity policy above).  BLS_INLINE_PRODUCTS=1 inlines
// the bodies instead (bigger code, slower compiles; for experiments).
#if defined(__HIP_DEVICE_COMPILE__) && !BLS_INLINE_PRODUCTS
struct fp_ret {
  uint32_t l[BLS_NL];
};
#define BLS_ARGS14(x) \
  x.l[0], x.l[1], x.l[2], x.l[3], x.l[4], x.l[5], x.l[6], x.l[7], x.l[8], x.l[9], x.l[10], x.l[11], x.l[12], x.l[13]
#define BLS_PARAMS14(x)                                                                                     \
  uint32_t x##0, uint32_t x##1, uint32_t x##2, uint32_t x##3, uint32_t x##4, uint32_t x##5, uint32_t x##6, \
      uint32_t x##7, uint32_t x##8, uint32_t x##9, uint32_t x##10, uint32_t x##11, uint32_t x##12, uint32_t x##13
#define BLS_INIT14(x) {{x##0, x##1, x##2, x##3, x##4, x##5, x##6, x##7, x##8, x##9, x##10, x##11, x##12, x##13}}
__device__ __noinline__ fp_ret fp_mul_r(BLS_PARAMS14(a), BLS_PARAMS14(b)) {
  const fp x = BLS_INIT14(a), y = BLS_INIT14(b);
  const fp r = fp_mul_body(x, y);
  fp_ret o;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) o.l[i] = r.l[i];
  return o;
}
__device__ __noinline__ fp_ret fp_sqr_r(BLS_PARAMS14(a)) {
  const fp x = BLS_INIT14(a);
  const fp r = fp_sqr_body(x);
  fp_ret o;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) o.l[i] = r.l[i];
  return o;
}
__device__ __forceinline__ fp fp_mul(const fp& a, const fp& b) {
  const fp_ret t = fp_mul_r(BLS_ARGS14(a), BLS_ARGS14(b));
  fp r;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) r.l[i] = t.l[i];
  return r;
}
__device__ __forceinline__ fp fp_sqr(const fp& a) {
  const fp_ret t = fp_sqr_r(BLS_ARGS14(a));
  fp r;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) r.l[i] = t.l[i];
  return r;
}
#else
BLS_INL fp fp_mul(const fp& a, const fp& b) {
  BLS_COUNT(bls_count_mul);
  return fp_mul_body(a, b);
}
BLS_INL fp fp_sqr(const fp& a) {
  BLS_COUNT(bls_count_sqr);
  return fp_sqr_body(a);
}
#endif

// ------------------------------------------------------------------------------------------------
// Additive operations (keep value <= 2p, limbs normalized)
// ------------------------------------------------------------------------------------------------
// s (value <= 4p, normalized) -> s or s - 2p
BLS_HD fp fp_csub_2p(const fp& s) {
  fp t;
  int32_t bw = 0;
#pragma unroll
  for (int i = 0; i < BLS_NL - 1; i++) {
    int32_t v = (int32_t)s.l[i] - (int32_t)FP_2P.l[i] + bw;
    t.l[i] = (uint32_t)v & BLS_MASK;
    bw = v >> BLS_LB;
  }
  int32_t top = (int32_t)s.l[BLS_NL - 1] - (int32_t)FP_2P.l[BLS_NL - 1] + bw;
  t.l[BLS_NL - 1] = (uint32_t)top;
  const bool neg = top < 0;
  fp r;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) r.l[i] = neg ? s.l[i] : t.l[i];
  return r;
}

BLS_HD fp fp_add(const fp& a, const fp& b) {
  fp s;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < BLS_NL - 1; i++) {
    uint32_t v = a.l[i] + b.l[i] + c;
    s.l[i] = v & BLS_MASK;
    c = v >> BLS_LB;
  }
  s.l[BLS_NL - 1] = a.l[BLS_NL - 1] + b.l[BLS_NL - 1] + c;
  return fp_csub_2p(s);
}

// Un-normalized, un-reduced sum: only as an operand of fp_mul / fp_sqr (see header comment).
BLS_HD fp fp_add_nr(const fp& a, const fp& b) {
  fp s;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) s.l[i] = a.l[i] + b.l[i];
  return s;
}

// a + b with the carries propagated but no reduction: normalized limbs, value <= a + b (an operand-side sum)
BLS_HD fp fp_add_norm(const fp& a, const fp& b) {
  fp s;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < BLS_NL - 1; i++) {
    uint32_t v = a.l[i] + b.l[i] + c;
    s.l[i] = v & BLS_MASK;
    c = v >> BLS_LB;
  }
  s.l[BLS_NL - 1] = a.l[BLS_NL - 1] + b.l[BLS_NL - 1] + c;
  return s;
}

// 8p with every limb but the top borrowed up into [2^28 - 1, 2^29): a + FP_8P_K - b has no negative limb for any
// normalized b of value <= 4p (its top limb stays below FP_8P_K's) -- the lazy subtraction below
BLS_CONST fp FP_8P_K = {{0x1ffd5558, 0x1f7ffffe, 0x1ffffdce, 0x1fff58a8, 0x1120f55e, 0x107b587a, 0x1b398694, 0x19c2895e, 0x13ba5c26, 0x15d66bb1, 0x1d3db219, 0x134d258c, 0x1f51cbfe, 0x000d0087}};
// a - b (mod p) as a lazy fp_mul operand: a + 8p - b limb by limb, no carries, no reduction.  a: limbs < 2^29;
// b: normalized, value <= 4p.  Result: limbs < 2^30, value < a + 8p (only as an operand of fp_mul, whose column sums
// and output bound allow limbs < 2^30 and values < 16p -- never stored).
BLS_HD fp fp_sub_k8(const fp& a, const fp& b) {
  fp s;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) s.l[i] = a.l[i] + FP_8P_K.l[i] - b.l[i];
  return s;
}

BLS_HD fp fp_sub(const fp& a, const fp& b) {
  // a + 2p - b  in [0, 4p]  -> conditional subtract 2p
  fp s;
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < BLS_NL - 1; i++) {
    int32_t v = (int32_t)a.l[i] + (int32_t)FP_2P.l[i] - (int32_t)b.l[i] + c;
    s.l[i] = (uint32_t)v & BLS_MASK;
    c = v >> BLS_LB;
  }
  s.l[BLS_NL - 1] = (uint32_t)((int32_t)a.l[BLS_NL - 1] + (int32_t)FP_2P.l[BLS_NL - 1] - (int32_t)b.l[BLS_NL - 1] + c);
  return fp_csub_2p(s);
}

BLS_HD fp fp_neg(const fp& a) {
  // 2p - a in [0, 2p]
  fp s;
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < BLS_NL - 1; i++) {
    int32_t v = (int32_t)FP_2P.l[i] - (int32_t)a.l[i] + c;
    s.l[i] = (uint32_t)v & BLS_MASK;
    c = v >> BLS_LB;
  }
  s.l[BLS_NL - 1] = (uint32_t)((int32_t)FP_2P.l[BLS_NL - 1] - (int32_t)a.l[BLS_NL - 1] + c);
  return s;
}

BLS_HD fp fp_dbl(const fp& a) { return fp_add(a, a); }

// a / 2 (mod p): make even by adding p when odd, then shift right one bit.
BLS_HD fp fp_half(const fp& a) {
  const uint32_t odd = 0u - (a.l[0] & 1u);
  fp s;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < BLS_NL - 1; i++) {
    uint32_t v = a.l[i] + (FP_P.l[i] & odd) + c;
    s.l[i] = v & BLS_MASK;
    c = v >> BLS_LB;
  }
  s.l[BLS_NL - 1] = a.l[BLS_NL - 1] + (FP_P.l[BLS_NL - 1] & odd) + c;  // value <= 3p
  fp r;
#pragma unroll
  for (int i = 0; i < BLS_NL - 1; i++) r.l[i] = (s.l[i] >> 1) | ((s.l[i + 1] & 1u) << (BLS_LB - 1));
  r.l[BLS_NL - 1] = s.l[BLS_NL - 1] >> 1;
  return r;  // value <= 1.5p
}

// small multiples (value <= 2p in, <= 2p out)
BLS_HD fp fp_mul3(const fp& a) { return fp_add(fp_dbl(a), a); }
BLS_HD fp fp_mul4(const fp& a) { return fp_dbl(fp_dbl(a)); }
BLS_HD fp fp_mul8(const fp& a) { return fp_dbl(fp_mul4(a)); }

BLS_HD fp fp_zero() {
  fp r;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) r.l[i] = 0;
  return r;
}
BLS_HD fp fp_one() { return FP_ONE; }

// Canonical representative in [0, p)
BLS_HD fp fp_csub_p(const fp& s) {
  fp t;
  int32_t bw = 0;
#pragma unroll
  for (int i = 0; i < BLS_NL - 1; i++) {
    int32_t v = (int32_t)s.l[i] - (int32_t)FP_P.l[i] + bw;
    t.l[i] = (uint32_t)v & BLS_MASK;
    bw = v >> BLS_LB;
  }
  int32_t top = (int32_t)s.l[BLS_NL - 1] - (int32_t)FP_P.l[BLS_NL - 1] + bw;
  t.l[BLS_NL - 1] = (uint32_t)top;
  const bool neg = top < 0;
  fp r;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) r.l[i] = neg ? s.l[i] : t.l[i];
  return r;
}
BLS_HD fp fp_canon(const fp& a) { return fp_csub_p(fp_csub_p(a)); }

// ------------------------------------------------------------------------------------------------
// Lazily reduced linear combinations: fp_lc(T<w>(x), ...) = sum w_k x_k (mod p), reduced ONCE.
//
// The additive glue of the tower and point formulas (t0 + xi (X - t1 - t2), ...) is where a chain of fp_add / fp_sub
// spends ~90 instructions per operation (carry pass + conditional 2p subtraction).  Here every term is added or
// subtracted limb by limb in uint32 without carries, on top of a multiple K p of p whose lower 13 limbs are raised to
// >= N (2^28 - 1) by borrowing (N = total negative weight), so no limb ever goes negative; then ONE pass subtracts
// q p for a floor estimate q of value / p (from the top two limbs) while propagating the carries.
// Terms: normalized limbs (< 2^28, top limb < 2^28) and values <= 2p (stored values, product outputs).  Weights
// w in [-15, 15], total |w| <= 15 (limb sums stay below 2^32).  Result: normalized, value in [0, 1.003 p).
// ------------------------------------------------------------------------------------------------
struct lc_limbs {
  uint32_t l[BLS_NL];
};
// K p (K = 2N: covers N negative unit terms of value <= 2p) in borrowed form: limb 0 + N 2^28, limbs 1..12 + N 2^28 -
// N, limb 13 - N (the value is unchanged, limbs 0..12 end up >= N (2^28 - 1)).
constexpr lc_limbs lc_ofs(int N) {
  lc_limbs r{};
  uint64_t c = 0;
  for (int i = 0; i < BLS_NL; i++) {
    const uint64_t v = (uint64_t)FP_P.l[i] * (uint64_t)(2 * N) + c;
    r.l[i] = i < BLS_NL - 1 ? (uint32_t)(v & BLS_MASK) : (uint32_t)v;
    c = v >> BLS_LB;
  }
  for (int i = 0; i < BLS_NL; i++) {
    if (i < BLS_NL - 1) r.l[i] += (uint32_t)N << BLS_LB;
    if (i > 0) r.l[i] -= (uint32_t)N;
  }
  return r;
}
template <int N>
struct LcOfs {
  static constexpr lc_limbs v = lc_ofs(N);
};
template <int W>
struct lc_term {
  const fp& x;
};
template <int W>
BLS_HD lc_term<W> T(const fp& x) {
  return lc_term<W>{x};
}
template <int W>
BLS_HD void lc_apply(uint32_t* s, const lc_term<W>& t) {
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) {
    if (W > 0)
      s[i] += (uint32_t)W * t.x.l[i];
    else
      s[i] -= (uint32_t)(-W) * t.x.l[i];
  }
}
template <int W>
constexpr int lc_neg_w() {
  return W < 0 ? -W : 0;
}
template <int W>
constexpr int lc_abs_w() {
  return W < 0 ? -W : W;
}
// NP = 2^392 - p in 28-bit limbs (limb 0: 2^28 - p_0, limbs 1..13: 2^28 - 1 - p_i)
constexpr lc_limbs lc_np() {
  lc_limbs r{};
  for (int i = 0; i < BLS_NL; i++) r.l[i] = (i == 0 ? (1u << BLS_LB) : BLS_MASK) - FP_P.l[i];
  return r;
}
BLS_CONST lc_limbs LC_NP = lc_np();
// s: limbs 0..12 unsigned (< 2^32), limb 13 signed; value = sum s_i 2^(28 i) >= 0 and < 64 p
BLS_HD fp lc_reduce(const uint32_t* s) {
  // q = floor((s13 2^28 + s12) 10080 / 2^58), 10080 = floor(2^394 / p): never above floor(value / p) (the limbs
  // below 12 add < 2^340 and only raise the value), at most 1 below (reciprocal error 8.3e-5 relative) -> the
  // result value is in [0, 1.003 p).  A negative top (value < 2^368) gives q = 0.
  const int64_t vhi = (int64_t)(int32_t)s[BLS_NL - 1] * (int64_t)(1u << BLS_LB) + (int64_t)s[BLS_NL - 2];
  const int32_t q = (int32_t)((uint64_t)(vhi > 0 ? vhi : 0) * 10080ull >> 58);
  // v - q p = v + q (2^392 - p) - q 2^392: unsigned MADs with the limbs of NP = 2^392 - p (all in [0, 2^28)), the q 2^392
  // leaving through the top limb (signed there).  Plain C: the same code on the device and in the host build.
  fp r;
  uint64_t acc = 0;
#pragma unroll
  for (int i = 0; i < BLS_NL - 1; i++) {
    acc = (acc >> BLS_LB) + (uint64_t)s[i] + (uint64_t)(uint32_t)q * (uint64_t)LC_NP.l[i];
    r.l[i] = (uint32_t)acc & BLS_MASK;
  }
  r.l[BLS_NL - 1] = (uint32_t)((int64_t)(acc >> BLS_LB) + (int64_t)(int32_t)s[BLS_NL - 1] -
                               (int64_t)q * (int64_t)(FP_P.l[BLS_NL - 1] + 1));
  return r;
}
template <int... W>
BLS_HD fp fp_lc(const lc_term<W>&... t) {
  constexpr int N = (0 + ... + lc_neg_w<W>());
  static_assert((0 + ... + lc_abs_w<W>()) <= 15, "fp_lc: total weight <= 15");
  uint32_t s[BLS_NL];
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) s[i] = LcOfs<N>::v.l[i];
  (lc_apply(s, t), ...);
  return lc_reduce(s);
}

BLS_HD bool fp_is_zero(const fp& a) {
  fp c = fp_canon(a);
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) o |= c.l[i];
  return o == 0;
}

BLS_HD bool fp_eq(const fp& a, const fp& b) { return fp_is_zero(fp_sub(a, b)); }

BLS_HD fp fp_select(bool c, const fp& a, const fp& b) {
  fp r;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) r.l[i] = c ? a.l[i] : b.l[i];
  return r;
}

// Montgomery conversions
BLS_HD fp fp_to_mont(const fp& plain) { return fp_mul(plain, FP_R2); }
BLS_HD fp fp_from_mont(const fp& a) {
  fp one = fp_zero();
  one.l[0] = 1;
  return fp_canon(fp_mul(a, one));
}

// Exponentiation by a public constant: left-to-right sliding window of width 4 over the odd powers
// a, a^3, ..., a^15 (379-381-bit exponents: 378 squarings + ~79 multiplications + 8 for the table, against
// 378 + ~228 for the binary method).  Every branch depends only on the public, wave-uniform exponent.  The
// table is a private array indexed by the (uniform) window digit: the same window with the eight powers held
// as separate named values across the product calls and picked by a switch produced wrong results on gfx950
// in the STAGE_KERNEL translation units (hipcc 7.2; tests/test_gpu_* caught it), the array form and a
// width-3 window are correct -- keep it this way.  BLS_BINARY_POW=1 restores the binary method.
#if BLS_BINARY_POW
BLS_HDNI fp fp_pow_words(const fp& a, const uint32_t* e, int nbits) {
  fp r = a;
  for (int i = nbits - 2; i >= 0; i--) {
    r = fp_sqr(r);
    if ((e[i >> 5] >> (i & 31)) & 1u) r = fp_mul(r, a);
  }
  return r;
}
#else
// The chain is one dependent product after another, so the products are inlined here (BLS_POW_INLINE, default
// on device): no call boundary per product (+26% products/s for a dependent chain at one wave per SIMD,
// profiles/r02_ilp_rate.json inl1 vs call1) for the cost of one squaring and one multiplication body of code.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(BLS_POW_INLINE)
#define BLS_POW_INLINE 1
#endif
#if BLS_POW_INLINE
#define BLS_POW_SQR(x) fp_sqr_body(x)
#define BLS_POW_MUL(x, y) fp_mul_body(x, y)
#else
#define BLS_POW_SQR(x) fp_sqr(x)
#define BLS_POW_MUL(x, y) fp_mul(x, y)
#endif
BLS_HDNI fp fp_pow_words(const fp& a, const uint32_t* e, int nbits) {
  fp tab[8];
  const fp a2 = fp_sqr(a);
  tab[0] = a;
  for (int k = 1; k < 8; k++) tab[k] = fp_mul(tab[k - 1], a2);
  fp r = a;
  bool started = false;
  int i = nbits - 1;
  while (i >= 0) {
    if (!((e[i >> 5] >> (i & 31)) & 1u)) {
      r = BLS_POW_SQR(r);
      i--;
      continue;
    }
    int j = i - 3 < 0 ? 0 : i - 3;
    while (!((e[j >> 5] >> (j & 31)) & 1u)) j++;
    uint32_t d = 0;
    for (int k = i; k >= j; k--) d = (d << 1) | ((e[k >> 5] >> (k & 31)) & 1u);
    if (started) {
      // the table entry is read before the window's squarings, so its (scratch) load latency hides behind them
      const fp t = tab[d >> 1];
      for (int k = i; k >= j; k--) r = BLS_POW_SQR(r);
      r = BLS_POW_MUL(r, t);
    } else {
      r = tab[d >> 1];
      started = true;
    }
    i = j - 1;
  }
  return r;
}
#endif

BLS_HD fp fp_inv_pow(const fp& a) { return fp_pow_words(a, EXP_P_MINUS_2, 381); }   // 0 -> 0

// ------------------------------------------------------------------------------------------------
// Inversion by Bernstein-Yang divsteps ("safegcd", eprint 2019/266): the extended binary gcd of p and the canonical
// value x of the element, in batches of 28 divsteps whose 2x2 transition matrix is found from the low 32 bits of
// f, g alone and then applied to the full-width f, g and to the Bezout coefficients d, e (kept mod p by adding the
// multiple of p that makes each batch's division by 2^28 exact -- a one-limb Montgomery step).  The control flow
// does not depend on the data (a fixed 40 batches: the paper's bound floor((49 * 381 + 57) / 17) = 1101 divsteps for
// 381-bit inputs), so the 64 lanes of a wave stay converged.  ~40k 32-bit VALU operations against ~460 Montgomery
// products (~210k instructions) for x^(p-2): an inversion on a latency-critical lane (the final exponentiation's,
// the batched affine conversions') costs a tenth of the exponentiation.
// Invariants: f = d x, g = e x (mod p); at the end g = 0 and f = +-1, so x^-1 = f d.  Multi-limb signed values: 14
// limbs, 0..12 in [0, 2^28), limb 13 a signed int32 (two's-complement top).
// ------------------------------------------------------------------------------------------------
#define BLS_BY_BATCHES 40
#define BLS_BY_STEPS 28

// (u a + v b) / 2^28 (exact: the caller's low 28 bits vanish) and, with `modp`, plus m p for the m that makes them
// vanish; a, b, out: signed 14-limb values (out may alias a or b)
BLS_INL void by_lincomb(const int32_t* a, const int32_t* b, int32_t u, int32_t v, bool modp, int32_t* out) {
  int64_t acc = (int64_t)u * a[0] + (int64_t)v * b[0];
  int32_t m = 0;
  if (modp) {
    m = (int32_t)(((uint32_t)acc * BLS_N0INV) & BLS_MASK);
    acc += (int64_t)m * (int64_t)FP_P.l[0];
  }
  acc >>= BLS_LB;  // the low 28 bits are zero
  int32_t o[BLS_NL];
#pragma unroll
  for (int j = 1; j < BLS_NL; j++) {
    acc += (int64_t)u * a[j] + (int64_t)v * b[j];
    if (modp) acc += (int64_t)m * (int64_t)FP_P.l[j];
    o[j - 1] = (int32_t)((uint32_t)acc & BLS_MASK);
    acc >>= BLS_LB;
  }
  o[BLS_NL - 1] = (int32_t)acc;
#pragma unroll
  for (int j = 0; j < BLS_NL; j++) out[j] = o[j];
}

BLS_HDNI fp fp_inv(const fp& a) {  // 0 -> 0
  const fp x = fp_canon(a);
  int32_t F[BLS_NL], G[BLS_NL], D[BLS_NL], E[BLS_NL];
#pragma unroll
  for (int j = 0; j < BLS_NL; j++) {
    F[j] = (int32_t)FP_P.l[j];
    G[j] = (int32_t)x.l[j];
    D[j] = 0;
    E[j] = 0;
  }
  E[0] = 1;
  int32_t delta = 1;
#pragma unroll 1
  for (int bt = 0; bt < BLS_BY_BATCHES; bt++) {
    // low 32 bits of f and g (limb 0 + the low 4 bits of limb 1): exact enough for 28 divsteps
    uint32_t f = (uint32_t)F[0] | ((uint32_t)F[1] << BLS_LB), g = (uint32_t)G[0] | ((uint32_t)G[1] << BLS_LB);
    int32_t u = 1, v = 0, q = 0, r = 1;  // [f; g] 2^i = [u v; q r] [f0; g0] over the batch
#pragma unroll
    for (int i = 0; i < BLS_BY_STEPS; i++) {
      // delta > 0 and g odd: (f, g, row f, row g) <- (g, -f, row g, -row f), delta <- -delta
      const bool sw = delta > 0 && (g & 1u);
      const uint32_t f0 = f;
      const int32_t u0 = u, v0 = v;
      f = sw ? g : f;
      g = sw ? 0u - f0 : g;
      u = sw ? q : u;
      v = sw ? r : v;
      q = sw ? -u0 : q;
      r = sw ? -v0 : r;
      delta = sw ? -delta : delta;
      // g odd: g += f, row g += row f  (then g is even)
      const uint32_t odd = 0u - (g & 1u);
      g += f & odd;
      q += u & (int32_t)odd;
      r += v & (int32_t)odd;
      // g /= 2 (row f doubles in the 2^i scaling)
      delta += 1;
      g >>= 1;
      u = (int32_t)((uint32_t)u << 1);  // (left shifts of negative ints are undefined in C++17)
      v = (int32_t)((uint32_t)v << 1);
    }
    int32_t nF[BLS_NL], nD[BLS_NL];
    by_lincomb(F, G, u, v, false, nF);
    by_lincomb(F, G, q, r, false, G);
    by_lincomb(D, E, u, v, true, nD);
    by_lincomb(D, E, q, r, true, E);
#pragma unroll
    for (int j = 0; j < BLS_NL; j++) {
      F[j] = nF[j];
      D[j] = nD[j];
    }
  }
  // f = +-1 (or p when x = 0, where d = 0): x^-1 = f d; |d| < 41 p, so f d + 42 p is a positive normalized value < 83 p
  const bool neg = F[BLS_NL - 1] < 0;
  fp y;
  int64_t c = 0;
#pragma unroll
  for (int j = 0; j < BLS_NL; j++) {
    c += (int64_t)(neg ? -(int64_t)D[j] : (int64_t)D[j]) + 42 * (int64_t)FP_P.l[j];
    if (j < BLS_NL - 1) {
      y.l[j] = (uint32_t)c & BLS_MASK;
      c >>= BLS_LB;
    } else {
      y.l[j] = (uint32_t)c;
    }
  }
  // y = (aR)^-1 mod p in plain form; the Montgomery form of a^-1 is y R^2 = Mont(y, R^3) (output < 1.05 p)
  return fp_mul(y, FP_R3);
}
BLS_HD fp fp_pow_p34(const fp& a) { return fp_pow_words(a, EXP_P_MINUS_3_DIV_4, 379); }

// Big-endian 48-byte <-> canonical integer limbs (not Montgomery).  Returns false if value >= p.
BLS_HD bool fp_from_be48_plain(const uint8_t* b, fp& out, uint8_t top_mask) {
  // bits: byte b[47 - j] holds bits 8j..8j+7
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) out.l[i] = 0;
#pragma unroll
  for (int j = 0; j < 48; j++) {
    uint32_t byte = b[47 - j];
    if (j == 47) byte &= top_mask;
    int bit = 8 * j;
    int li = bit / BLS_LB, off = bit % BLS_LB;
    out.l[li] |= (byte << off) & BLS_MASK;
    if (off > BLS_LB - 8 && li + 1 < BLS_NL) out.l[li + 1] |= byte >> (BLS_LB - off);
  }
  // compare with p
  int32_t bw = 0;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) {
    int32_t v = (int32_t)out.l[i] - (int32_t)FP_P.l[i] + bw;
    bw = v >> BLS_LB;
  }
  return bw < 0;  // value < p
}

BLS_HD void fp_to_be48_plain(const fp& canon, uint8_t* b) {
#pragma unroll
  for (int j = 0; j < 48; j++) {
    int bit = 8 * j;
    int li = bit / BLS_LB, off = bit % BLS_LB;
    uint32_t v = canon.l[li] >> off;
    if (off > BLS_LB - 8 && li + 1 < BLS_NL) v |= canon.l[li + 1] << (BLS_LB - off);
    b[47 - j] = (uint8_t)v;
  }
}

// value > (p-1)/2 for a canonical plain value  (ZCash "lexicographically largest")
BLS_HD bool fp_plain_gt_half(const fp& canon) {
  // compute 2*v - p: v > (p-1)/2  <=>  2v > p - 1  <=>  2v >= p
  int32_t bw = 0;
  uint32_t carry = 0;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) {
    uint32_t d = (canon.l[i] << 1) + carry;
    carry = d >> BLS_LB;
    if (i < BLS_NL - 1) d &= BLS_MASK;
    int32_t v = (int32_t)d - (int32_t)FP_P.l[i] + bw;
    bw = v >> BLS_LB;
  }
  return bw >= 0;
}

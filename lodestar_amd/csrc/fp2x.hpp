// Lane-pair Fp2 ("fp2x"): lanes 2j and 2j + 1 of a wave hold coefficients c0 and c1 of one Fp2 element, so a lane
// carries 14 registers per Fp2 value instead of 28.  The G2 point formulas of curve.hpp are written over a field type
// F; instantiated with fp2x they run one G2 point per lane pair with half the per-lane state -- small enough for two
// waves per SIMD without spills, where the one-lane form needs the whole 512-entry register file and a wave alone
// issues a v_mad_u64_u32 only every ~11 cycles against ~5.7 with two (profiles/r04_mad_mix.json).
//
// Products: each lane computes its own output coefficient as ONE Montgomery reduction of a two-term dot product,
//   lane 0:  c0 = Redc(a0 b0 + a1 (16p - b1))       (= a0 b0 - a1 b1 mod p, tower.hpp fp2_mul_sb_body's c0)
//   lane 1:  c1 = Redc(a1 b0 + a0 b1)
// i.e. Redc(a * B0 + a' * Y) with a' the partner's coefficient, B0 = b0 on both lanes and Y = 16p - b1 / b1 -- 588
// v_mad_u64_u32 per lane (the pair: the one-lane body's 1,176).  Squaring: c0 = (a0 + a1)(a0 + 8p - a1), c1 = (a0 +
// a0) a1, one product per lane (392).  The partner's limbs arrive by DPP row moves (quad_perm, no LDS).  Additive
// glue (add, sub, lazily reduced combinations) is coefficient-wise: each lane runs the Fp operation on its own
// coefficient.  Lane pairs are always active together (kernels exit per pair), and every branch condition the point
// formulas take (F_is_zero) is combined over the pair, so both lanes follow the same path.
#pragma once
#include "curve.hpp"

struct fp2x {
  fp v;
};
typedef jac<fp2x> g2jx;

#if defined(__HIP_DEVICE_COMPILE__)
BLS_HD uint32_t fp2x_k() { return __lane_id() & 1u; }  // this lane's coefficient index
// partner / even / odd lane of the pair (DPP quad_perm [1,0,3,2] / [0,0,2,2] / [1,1,3,3])
BLS_HD uint32_t dpp_swap(uint32_t x) { return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false); }
BLS_HD uint32_t dpp_even(uint32_t x) { return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xA0, 0xF, 0xF, false); }
BLS_HD uint32_t dpp_odd(uint32_t x) { return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xF5, 0xF, 0xF, false); }
#else
// host build (tests/native/emu.cpp): a lane pair is emulated by the caller; not used
BLS_HD uint32_t fp2x_k() { return 0; }
BLS_HD uint32_t dpp_swap(uint32_t x) { return x; }
BLS_HD uint32_t dpp_even(uint32_t x) { return x; }
BLS_HD uint32_t dpp_odd(uint32_t x) { return x; }
#endif

BLS_HD fp fp_swap(const fp& x) {
  fp r;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) r.l[i] = dpp_swap(x.l[i]);
  return r;
}

// Redc(x1 y1 + x2 y2): product scanning of both products into one accumulator, one reduction.  Operands: limbs of x1,
// x2, y1 < 2^29 and of y2 < 2^30 (the 16p - b1 offset form); column bound 14 (2^58 + 2^59) + 14 * 2^56 + 2^36 < 2^64
// (fp2_mul_sb_body's c0).  Output: normalized limbs, value < 1.1 p for operand values < 8p (y2 < 16p + 8p).
BLS_INL fp fp_dot_body(const fp& x1, const fp& y1, const fp& x2, const fp& y2) {
  uint32_t m[BLS_NL];
  uint64_t acc = 0;
  fp r;
#pragma unroll
  for (int k = 0; k < 2 * BLS_NL - 1; k++) {
    const int lo = k < BLS_NL ? 0 : k - BLS_NL + 1, hi = k < BLS_NL ? k : BLS_NL - 1;
#pragma unroll
    for (int i = lo; i <= hi; i++) {
      acc += (uint64_t)x1.l[i] * y1.l[k - i];
      acc += (uint64_t)x2.l[i] * y2.l[k - i];
    }
    const int mhi = k < BLS_NL ? k - 1 : BLS_NL - 1;
#pragma unroll
    for (int i = lo; i <= mhi; i++) acc += (uint64_t)m[i] * FP_P.l[k - i];
    if (k < BLS_NL) {
      const uint32_t q = ((uint32_t)acc * BLS_N0INV) & BLS_MASK;
      m[k] = q;
      acc += (uint64_t)q * FP_P.l[0];
    } else {
      r.l[k - BLS_NL] = (uint32_t)acc & BLS_MASK;
    }
    acc >>= BLS_LB;
  }
  r.l[BLS_NL - 1] = (uint32_t)acc;
  return r;
}

// this lane's coefficient of a * b.  a, b: limbs < 2^29, values < 8p (normalized values or one fp_add_nr level)
BLS_INL fp fp2x_mul_body(const fp& a, const fp& b) {
  const bool odd = fp2x_k() != 0;
  fp pa, b0, y;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) {
    pa.l[i] = dpp_swap(a.l[i]);
    b0.l[i] = dpp_even(b.l[i]);
    const uint32_t b1 = dpp_odd(b.l[i]);
    y.l[i] = odd ? b1 : FP_16P_K.l[i] - b1;
  }
  return fp_dot_body(a, b0, pa, y);
}
// this lane's coefficient of a^2.  a: normalized limbs, value <= 4p (tower.hpp fp2_sqr_body's contract)
BLS_INL fp fp2x_sqr_body(const fp& a) {
  const bool odd = fp2x_k() != 0;
  fp x, y;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) {
    const uint32_t a0 = dpp_even(a.l[i]), a1 = dpp_odd(a.l[i]);
    x.l[i] = a0 + (odd ? a0 : a1);
    y.l[i] = odd ? a1 : a0 + FP_8P_K.l[i] - a1;
  }
  return fp_mul_body(x, y);
}

#if defined(__HIP_DEVICE_COMPILE__) && !BLS_INLINE_PRODUCTS
// register-ABI calls (fp.hpp call-granularity policy): 28 / 14 VGPR arguments, 14 returned
__device__ __noinline__ fp_ret fp2x_mul_r(BLS_PARAMS14(a), BLS_PARAMS14(b)) {
  const fp x = BLS_INIT14(a), y = BLS_INIT14(b);
  const fp r = fp2x_mul_body(x, y);
  fp_ret o;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) o.l[i] = r.l[i];
  return o;
}
__device__ __noinline__ fp_ret fp2x_sqr_r(BLS_PARAMS14(a)) {
  const fp x = BLS_INIT14(a);
  const fp r = fp2x_sqr_body(x);
  fp_ret o;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) o.l[i] = r.l[i];
  return o;
}
__device__ __forceinline__ fp2x fp2x_mul(const fp2x& a, const fp2x& b) {
  const fp_ret t = fp2x_mul_r(BLS_ARGS14(a.v), BLS_ARGS14(b.v));
  fp2x r;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) r.v.l[i] = t.l[i];
  return r;
}
__device__ __forceinline__ fp2x fp2x_sqr(const fp2x& a) {
  const fp_ret t = fp2x_sqr_r(BLS_ARGS14(a.v));
  fp2x r;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) r.v.l[i] = t.l[i];
  return r;
}
#else
BLS_INL fp2x fp2x_mul(const fp2x& a, const fp2x& b) { return fp2x{fp2x_mul_body(a.v, b.v)}; }
BLS_INL fp2x fp2x_sqr(const fp2x& a) { return fp2x{fp2x_sqr_body(a.v)}; }
#endif

// ---- the field interface of curve.hpp -------------------------------------------------------------
BLS_HD fp2x F_add(const fp2x& a, const fp2x& b) { return fp2x{fp_add(a.v, b.v)}; }
BLS_HD fp2x F_sub(const fp2x& a, const fp2x& b) { return fp2x{fp_sub(a.v, b.v)}; }
BLS_HD fp2x F_mul(const fp2x& a, const fp2x& b) { return fp2x_mul(a, b); }
BLS_HD fp2x F_sqr(const fp2x& a) { return fp2x_sqr(a); }
BLS_HD fp2x F_dbl(const fp2x& a) { return fp2x{fp_dbl(a.v)}; }
BLS_HD fp2x F_neg(const fp2x& a) { return fp2x{fp_neg(a.v)}; }
BLS_HD bool F_is_zero(const fp2x& a) {
  const uint32_t z = fp_is_zero(a.v) ? 1u : 0u;
  return (z & dpp_swap(z)) != 0;
}
BLS_HD fp2x F_select(bool c, const fp2x& a, const fp2x& b) { return fp2x{fp_select(c, a.v, b.v)}; }
BLS_HD fp2x F_add_nr(const fp2x& a, const fp2x& b) { return fp2x{fp_add_nr(a.v, b.v)}; }
BLS_HD fp2x F_add_sq(const fp2x& a, const fp2x& b) { return fp2x{fp_add_norm(a.v, b.v)}; }
template <int... W>
BLS_HD fp2x F_lc(const lt<W, fp2x>&... t) {
  return fp2x{fp_lc(T<W>(t.v.v)...)};
}
BLS_HD fp2x F_one(const fp2x*) { return fp2x{fp2x_k() ? fp_zero() : FP_ONE}; }
BLS_HD fp2x F_zero(const fp2x*) { return fp2x{fp_zero()}; }
template <>
struct lazy_curve<fp2x> {
  static constexpr bool dbl = BLS_LAZY_G2_DBL, add = BLS_LAZY_G2_ADD, addaff = BLS_LAZY_G2_ADDAFF;
};

// this lane's coefficient of an Fp2 constant / value
BLS_HD fp2x fp2x_of(const fp2& c) { return fp2x{fp2x_k() ? c.c1 : c.c0}; }
BLS_HD fp2x fp2x_conj(const fp2x& a) { return fp2x{fp2x_k() ? fp_neg(a.v) : a.v}; }

BLS_FN g2jx g2_psi(const g2jx& p) {
  g2jx r;
  r.x = fp2x_mul(fp2x_conj(p.x), fp2x_of(PSI_X));
  r.y = fp2x_mul(fp2x_conj(p.y), fp2x_of(PSI_Y));
  r.z = fp2x_conj(p.z);
  return r;
}
BLS_FN g2jx g2_psi2(const g2jx& p) {
  g2jx r;
  r.x = fp2x_mul(p.x, fp2x_of(PSI2_X));
  r.y = fp2x_mul(p.y, fp2x_of(PSI2_Y));
  r.z = p.z;
  return r;
}
// the pair's N(a) = a0^2 + a1^2 (both lanes)
BLS_FN fp fp2x_norm(const fp2x& a) {
  const fp s = fp_sqr(a.v);
  return fp_add(s, fp_swap(s));
}

// ---- Miller line steps on lane pairs (pairing.hpp miller_dbl_line / miller_add_line, the lazy forms) ---------
struct g2projx {
  fp2x x, y, z;
};
struct line3x {
  fp2x l0, c1, c4;
};
BLS_HD fp2x fp2x_half(const fp2x& a) { return fp2x{fp_half(a.v)}; }
// xi a = (a0 - a1) + (a0 + a1) u, this lane's coefficient (one lazily reduced combination)
BLS_FN fp2x fp2x_mul_xi(const fp2x& a) {
  const fp p = fp_swap(a.v);
  const fp d = fp_lc(T<1>(a.v), T<-1>(p)), s = fp_lc(T<1>(a.v), T<1>(p));
  return fp2x{fp2x_k() ? s : d};
}
BLS_FN void miller_dbl_line(g2projx& R, line3x& Ln) {
  const fp2x A = fp2x_half(F_mul(R.x, R.y));
  const fp2x B = F_sqr(R.y);
  const fp2x C = F_sqr(R.z);
  const fp2x E = F_lc(L<12>(fp2x_mul_xi(C)));
  const fp2x G = fp2x_half(F_lc(L<1>(B), L<3>(E)));
  const fp2x H = F_lc(L<1>(F_sqr(F_add_sq(R.y, R.z))), L<-1>(B), L<-1>(C));
  const fp2x J = F_sqr(R.x);
  const fp2x E2 = F_sqr(E);
  R.x = F_mul(A, F_lc(L<1>(B), L<-3>(E)));
  R.y = F_lc(L<1>(F_sqr(G)), L<-3>(E2));
  R.z = F_mul(B, H);
  Ln.l0 = F_lc(L<1>(E), L<-1>(B));
  Ln.c1 = F_lc(L<3>(J));
  Ln.c4 = F_lc(L<-1>(H));
}
BLS_FN void miller_add_line(g2projx& R, const aff<fp2x>& Q, line3x& Ln) {
  const fp2x theta = F_lc(L<1>(R.y), L<-1>(F_mul(Q.y, R.z)));
  const fp2x lam = F_lc(L<1>(R.x), L<-1>(F_mul(Q.x, R.z)));
  const fp2x C = F_sqr(theta);
  const fp2x D = F_sqr(lam);
  const fp2x E = F_mul(lam, D);
  const fp2x Fv = F_mul(R.z, C);
  const fp2x G = F_mul(R.x, D);
  const fp2x H = F_lc(L<1>(E), L<1>(Fv), L<-2>(G));
  const fp2x X3 = F_mul(lam, H);
  const fp2x Y3 = F_lc(L<1>(F_mul(theta, F_lc(L<1>(G), L<-1>(H)))), L<-1>(F_mul(R.y, E)));
  const fp2x Z3 = F_mul(R.z, E);
  Ln.l0 = F_lc(L<1>(F_mul(theta, Q.x)), L<-1>(F_mul(lam, Q.y)));
  Ln.c1 = F_lc(L<-1>(theta));
  Ln.c4 = lam;
  R.x = X3;
  R.y = Y3;
  R.z = Z3;
}

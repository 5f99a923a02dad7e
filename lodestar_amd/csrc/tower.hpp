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

BLS_FN fp2 fp2_mul(const fp2& a, const fp2& b) {
  fp t0 = fp_mul(a.c0, b.c0);
  fp t1 = fp_mul(a.c1, b.c1);
  fp t2 = fp_mul(fp_add_nr(a.c0, a.c1), fp_add_nr(b.c0, b.c1));
  return fp2_make(fp_sub(t0, t1), fp_sub(fp_sub(t2, t0), t1));
}

BLS_FN fp2 fp2_sqr(const fp2& a) {
  fp c0 = fp_mul(fp_add_nr(a.c0, a.c1), fp_sub(a.c0, a.c1));
  fp c1 = fp_mul(fp_add_nr(a.c0, a.c0), a.c1);
  return fp2_make(c0, c1);
}

BLS_FN fp2 fp2_mul_fp(const fp2& a, const fp& s) { return fp2_make(fp_mul(a.c0, s), fp_mul(a.c1, s)); }

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

BLS_FN fp6 fp6_mul(const fp6& a, const fp6& b) {
  fp2 t0 = fp2_mul(a.c0, b.c0);
  fp2 t1 = fp2_mul(a.c1, b.c1);
  fp2 t2 = fp2_mul(a.c2, b.c2);
  fp2 c0 = fp2_add(t0, fp2_mul_xi(fp2_sub(fp2_mul(fp2_add(a.c1, a.c2), fp2_add(b.c1, b.c2)), fp2_add(t1, t2))));
  fp2 c1 = fp2_add(fp2_sub(fp2_mul(fp2_add(a.c0, a.c1), fp2_add(b.c0, b.c1)), fp2_add(t0, t1)), fp2_mul_xi(t2));
  fp2 c2 = fp2_add(fp2_sub(fp2_mul(fp2_add(a.c0, a.c2), fp2_add(b.c0, b.c2)), fp2_add(t0, t2)), t1);
  return fp6_make(c0, c1, c2);
}

// (x0 + x1 v + x2 v^2)(l0 + l1 v)
BLS_FN fp6 fp6_mul_by_01(const fp6& x, const fp2& l0, const fp2& l1) {
  fp2 t0 = fp2_mul(x.c0, l0);
  fp2 t1 = fp2_mul(x.c1, l1);
  fp2 c0 = fp2_add(t0, fp2_mul_xi(fp2_mul(x.c2, l1)));
  fp2 c1 = fp2_sub(fp2_sub(fp2_mul(fp2_add(x.c0, x.c1), fp2_add(l0, l1)), t0), t1);
  fp2 c2 = fp2_add(fp2_mul(x.c2, l0), t1);
  return fp6_make(c0, c1, c2);
}

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

// --------------------------------------------------------------------------------------------- Fp12
BLS_HD fp12 fp12_make(const fp6& a, const fp6& b) {
  fp12 r;
  r.c0 = a;
  r.c1 = b;
  return r;
}
BLS_HD fp12 fp12_one() { return fp12_make(fp6_one(), fp6_zero()); }

BLS_FN fp12 fp12_mul(const fp12& a, const fp12& b) {
  fp6 t0 = fp6_mul(a.c0, b.c0);
  fp6 t1 = fp6_mul(a.c1, b.c1);
  fp6 c1 = fp6_sub(fp6_mul(fp6_add(a.c0, a.c1), fp6_add(b.c0, b.c1)), fp6_add(t0, t1));
  fp6 c0 = fp6_add(t0, fp6_mul_v(t1));
  return fp12_make(c0, c1);
}

// (a0 + a1 w)^2 = (a0^2 + v a1^2) + 2 a0 a1 w ;  complex-method squaring, 2 Fp6 muls
BLS_FN fp12 fp12_sqr(const fp12& a) {
  fp6 t = fp6_mul(a.c0, a.c1);
  fp6 s = fp6_mul(fp6_add(a.c0, a.c1), fp6_add(a.c0, fp6_mul_v(a.c1)));
  fp6 c0 = fp6_sub(fp6_sub(s, t), fp6_mul_v(t));
  fp6 c1 = fp6_add(t, t);
  return fp12_make(c0, c1);
}

BLS_HD fp12 fp12_conj(const fp12& a) { return fp12_make(a.c0, fp6_neg(a.c1)); }

BLS_BIG fp12 fp12_inv(const fp12& a) {
  fp6 t = fp6_sub(fp6_mul(a.c0, a.c0), fp6_mul_v(fp6_mul(a.c1, a.c1)));
  fp6 ti = fp6_inv(t);
  return fp12_make(fp6_mul(a.c0, ti), fp6_neg(fp6_mul(a.c1, ti)));
}

// f * line, line = l0 + l1 v + l4 v w   (positions c0.c0, c0.c1, c1.c1) -- 13 Fp2 multiplications
BLS_FN fp12 fp12_mul_by_014(const fp12& f, const fp2& l0, const fp2& l1, const fp2& l4) {
  fp6 a0 = fp6_mul_by_01(f.c0, l0, l1);
  fp6 a1 = fp6_mul_by_1(f.c1, l4);
  fp6 s = fp6_mul_by_01(fp6_add(f.c0, f.c1), l0, fp2_add(l1, l4));
  fp6 c1 = fp6_sub(fp6_sub(s, a0), a1);
  fp6 c0 = fp6_add(a0, fp6_mul_v(a1));
  return fp12_make(c0, c1);
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

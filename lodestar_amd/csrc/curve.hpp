// G1 (y^2 = x^3 + 4 over Fp) and G2 (y^2 = x^3 + 4(u+1) over Fp2) in Jacobian coordinates.
// Formulas: dbl-2009-l and madd/add-2007-bl (a = 0), with the exceptional cases (P = Q, P = -Q,
// infinity) handled by branches that only adversarial inputs take.
#pragma once
#include "tower.hpp"

// ---- field-generic wrappers so the point code is written once -----------------------------------
BLS_HD fp F_add(const fp& a, const fp& b) { return fp_add(a, b); }
BLS_HD fp F_sub(const fp& a, const fp& b) { return fp_sub(a, b); }
BLS_HD fp F_mul(const fp& a, const fp& b) { return fp_mul(a, b); }
BLS_HD fp F_sqr(const fp& a) { return fp_sqr(a); }
BLS_HD fp F_dbl(const fp& a) { return fp_dbl(a); }
BLS_HD fp F_neg(const fp& a) { return fp_neg(a); }
BLS_HD bool F_is_zero(const fp& a) { return fp_is_zero(a); }
BLS_HD fp F_select(bool c, const fp& a, const fp& b) { return fp_select(c, a, b); }
BLS_HD fp F_add_nr(const fp& a, const fp& b) { return fp_add_nr(a, b); }
// the operand-side sum a squaring takes: Fp one un-normalized level, Fp2 normalized (fp2_sqr's a0 - a1 needs limbs)
BLS_HD fp F_add_sq(const fp& a, const fp& b) { return fp_add_nr(a, b); }
BLS_HD fp2 F_add(const fp2& a, const fp2& b) { return fp2_add(a, b); }
BLS_HD fp2 F_sub(const fp2& a, const fp2& b) { return fp2_sub(a, b); }
BLS_HD fp2 F_mul(const fp2& a, const fp2& b) { return fp2_mul(a, b); }
BLS_HD fp2 F_sqr(const fp2& a) { return fp2_sqr(a); }
BLS_HD fp2 F_dbl(const fp2& a) { return fp2_dbl(a); }
BLS_HD fp2 F_neg(const fp2& a) { return fp2_neg(a); }
BLS_HD bool F_is_zero(const fp2& a) { return fp2_is_zero(a); }
BLS_HD fp2 F_select(bool c, const fp2& a, const fp2& b) { return fp2_select(c, a, b); }
BLS_HD fp2 F_add_nr(const fp2& a, const fp2& b) { return fp2_add_nr(a, b); }
BLS_HD fp2 F_add_sq(const fp2& a, const fp2& b) { return fp2_add_norm(a, b); }
// Lazily reduced linear combinations over either field (fp.hpp fp_lc; Fp2 component-wise): F_lc(L<w>(x), ...).
// Terms: normalized, values <= 2p (stored coordinates, products, F_lc results) -- never fp_add_nr sums.
template <int W, class F>
struct lt {
  const F& v;
};
template <int W, class F>
BLS_HD lt<W, F> L(const F& v) {
  return lt<W, F>{v};
}
template <int... W>
BLS_HD fp F_lc(const lt<W, fp>&... t) {
  return fp_lc(T<W>(t.v)...);
}
template <int... W>
BLS_HD fp2 F_lc(const lt<W, fp2>&... t) {
  return fp2_make(fp_lc(T<W>(t.v.c0)...), fp_lc(T<W>(t.v.c1)...));
}

template <class F>
struct jac {
  F x, y, z;
};
template <class F>
struct aff {
  F x, y;
};
typedef jac<fp> g1j;
typedef aff<fp> g1a;
typedef jac<fp2> g2j;
typedef aff<fp2> g2a;

BLS_HD fp F_one(const fp*) { return FP_ONE; }
BLS_HD fp2 F_one(const fp2*) { return fp2_one(); }
BLS_HD fp F_zero(const fp*) { return fp_zero(); }
BLS_HD fp2 F_zero(const fp2*) { return fp2_zero(); }

template <class F>
BLS_HD jac<F> jac_infinity() {
  jac<F> r;
  r.x = F_one((const F*)0);
  r.y = F_one((const F*)0);
  r.z = F_zero((const F*)0);
  return r;
}
template <class F>
BLS_HD bool jac_is_inf(const jac<F>& p) {
  return F_is_zero(p.z);
}
template <class F>
BLS_HD jac<F> jac_from_aff(const aff<F>& a) {
  jac<F> r;
  r.x = a.x;
  r.y = a.y;
  r.z = F_one((const F*)0);
  return r;
}

#ifndef BLS_LAZY_CURVE
#define BLS_LAZY_CURVE 1
#endif
// The additive glue as lazily reduced combinations (F_lc); X + B goes to the squaring as F_add_sq (value <= 4p, the
// squarings' operand contract).  D - X3 = 3 D - F.
template <class F>
BLS_FN jac<F> jac_dbl_lazy(const jac<F>& p) {
  const F A = F_sqr(p.x);
  const F B = F_sqr(p.y);
  const F C = F_sqr(B);
  const F S = F_sqr(F_add_sq(p.x, B));
  const F D = F_lc(L<2>(S), L<-2>(A), L<-2>(C));
  const F E = F_lc(L<3>(A));
  const F Fv = F_sqr(E);
  jac<F> r;
  r.x = F_lc(L<1>(Fv), L<-2>(D));
  const F M = F_mul(E, F_lc(L<3>(D), L<-1>(Fv)));
  r.y = F_lc(L<1>(M), L<-8>(C));
  r.z = F_mul(F_add_nr(p.y, p.y), p.z);
  return r;  // infinity (z = 0) maps to z = 0
}
template <class F>
BLS_FN jac<F> jac_dbl_eager(const jac<F>& p) {
  F A = F_sqr(p.x);
  F B = F_sqr(p.y);
  F C = F_sqr(B);
  F D = F_sub(F_sub(F_sqr(F_add(p.x, B)), A), C);
  D = F_dbl(D);
  F E = F_add(F_dbl(A), A);
  F Fv = F_sqr(E);
  jac<F> r;
  r.x = F_sub(Fv, F_dbl(D));
  F C8 = F_dbl(F_dbl(F_dbl(C)));
  r.y = F_sub(F_mul(E, F_sub(D, r.x)), C8);
  r.z = F_mul(F_add_nr(p.y, p.y), p.z);
  return r;  // infinity (z = 0) maps to z = 0
}
// lazy glue per group: BLS_LAZY_CURVE (both), BLS_LAZY_G1 / BLS_LAZY_G2 (one group)
#ifndef BLS_LAZY_G1
#define BLS_LAZY_G1 BLS_LAZY_CURVE
#endif
#ifndef BLS_LAZY_G2
#define BLS_LAZY_G2 BLS_LAZY_CURVE
#endif
#ifndef BLS_LAZY_G2_DBL
#define BLS_LAZY_G2_DBL BLS_LAZY_G2
#endif
#ifndef BLS_LAZY_G2_ADD
#define BLS_LAZY_G2_ADD BLS_LAZY_G2
#endif
#ifndef BLS_LAZY_G2_ADDAFF
#define BLS_LAZY_G2_ADDAFF BLS_LAZY_G2
#endif
template <class F>
struct lazy_curve {
  static constexpr bool dbl = BLS_LAZY_G1, add = BLS_LAZY_G1, addaff = BLS_LAZY_G1;
};
template <>
struct lazy_curve<fp2> {
  static constexpr bool dbl = BLS_LAZY_G2_DBL, add = BLS_LAZY_G2_ADD, addaff = BLS_LAZY_G2_ADDAFF;
};
template <class F>
BLS_FN jac<F> jac_dbl(const jac<F>& p) {
  if constexpr (lazy_curve<F>::dbl)
    return jac_dbl_lazy(p);
  else
    return jac_dbl_eager(p);
}

template <class F>
BLS_HD jac<F> jac_neg(const jac<F>& p) {
  jac<F> r = p;
  r.y = F_neg(p.y);
  return r;
}

// p + q with q affine (q never infinity here)
template <class F>
BLS_INL jac<F> jac_add_aff_lazy(const jac<F>& p, const aff<F>& q) {
  if (jac_is_inf(p)) return jac_from_aff(q);
  const F Z1Z1 = F_sqr(p.z);
  const F U2 = F_mul(q.x, Z1Z1);
  const F S2 = F_mul(q.y, F_mul(p.z, Z1Z1));
  const F H = F_lc(L<1>(U2), L<-1>(p.x));
  const F rr = F_lc(L<2>(S2), L<-2>(p.y));
  if (F_is_zero(H)) {
    if (F_is_zero(rr)) return jac_dbl(p);
    return jac_infinity<F>();
  }
  const F HH = F_sqr(H);
  const F I = F_lc(L<4>(HH));
  const F J = F_mul(H, I);
  const F V = F_mul(p.x, I);
  const F R2 = F_sqr(rr);
  jac<F> r;
  r.x = F_lc(L<1>(R2), L<-1>(J), L<-2>(V));
  const F M = F_mul(rr, F_lc(L<3>(V), L<-1>(R2), L<1>(J)));  // V - X3 = 3V - r^2 + J
  const F N = F_mul(p.y, J);
  r.y = F_lc(L<1>(M), L<-2>(N));
  r.z = F_lc(L<1>(F_sqr(F_add_sq(p.z, H))), L<-1>(Z1Z1), L<-1>(HH));
  return r;
}
template <class F>
BLS_INL jac<F> jac_add_aff_eager(const jac<F>& p, const aff<F>& q) {
  if (jac_is_inf(p)) return jac_from_aff(q);
  F Z1Z1 = F_sqr(p.z);
  F U2 = F_mul(q.x, Z1Z1);
  F S2 = F_mul(q.y, F_mul(p.z, Z1Z1));
  F H = F_sub(U2, p.x);
  F rr = F_dbl(F_sub(S2, p.y));
  if (F_is_zero(H)) {
    if (F_is_zero(rr)) return jac_dbl(p);
    return jac_infinity<F>();
  }
  F HH = F_sqr(H);
  F I = F_dbl(F_dbl(HH));
  F J = F_mul(H, I);
  F V = F_mul(p.x, I);
  jac<F> r;
  r.x = F_sub(F_sub(F_sqr(rr), J), F_dbl(V));
  r.y = F_sub(F_mul(rr, F_sub(V, r.x)), F_dbl(F_mul(p.y, J)));
  r.z = F_sub(F_sub(F_sqr(F_add(p.z, H)), Z1Z1), HH);
  return r;
}
template <class F>
BLS_INL jac<F> jac_add_aff(const jac<F>& p, const aff<F>& q) {
  if constexpr (lazy_curve<F>::addaff)
    return jac_add_aff_lazy(p, q);
  else
    return jac_add_aff_eager(p, q);
}

// general Jacobian addition
template <class F>
BLS_INL jac<F> jac_add_lazy(const jac<F>& p, const jac<F>& q) {
  if (jac_is_inf(p)) return q;
  if (jac_is_inf(q)) return p;
  const F Z1Z1 = F_sqr(p.z);
  const F Z2Z2 = F_sqr(q.z);
  const F U1 = F_mul(p.x, Z2Z2);
  const F U2 = F_mul(q.x, Z1Z1);
  const F S1 = F_mul(p.y, F_mul(q.z, Z2Z2));
  const F S2 = F_mul(q.y, F_mul(p.z, Z1Z1));
  const F H = F_lc(L<1>(U2), L<-1>(U1));
  const F rr = F_lc(L<2>(S2), L<-2>(S1));
  if (F_is_zero(H)) {
    if (F_is_zero(rr)) return jac_dbl(p);
    return jac_infinity<F>();
  }
  const F I = F_sqr(F_add_sq(H, H));
  const F J = F_mul(H, I);
  const F V = F_mul(U1, I);
  const F R2 = F_sqr(rr);
  jac<F> r;
  r.x = F_lc(L<1>(R2), L<-1>(J), L<-2>(V));
  const F M = F_mul(rr, F_lc(L<3>(V), L<-1>(R2), L<1>(J)));  // V - X3 = 3V - r^2 + J
  const F N = F_mul(S1, J);
  r.y = F_lc(L<1>(M), L<-2>(N));
  r.z = F_mul(F_lc(L<1>(F_sqr(F_add_sq(p.z, q.z))), L<-1>(Z1Z1), L<-1>(Z2Z2)), H);
  return r;
}
template <class F>
BLS_INL jac<F> jac_add_eager(const jac<F>& p, const jac<F>& q) {
  if (jac_is_inf(p)) return q;
  if (jac_is_inf(q)) return p;
  F Z1Z1 = F_sqr(p.z);
  F Z2Z2 = F_sqr(q.z);
  F U1 = F_mul(p.x, Z2Z2);
  F U2 = F_mul(q.x, Z1Z1);
  F S1 = F_mul(p.y, F_mul(q.z, Z2Z2));
  F S2 = F_mul(q.y, F_mul(p.z, Z1Z1));
  F H = F_sub(U2, U1);
  F rr = F_dbl(F_sub(S2, S1));
  if (F_is_zero(H)) {
    if (F_is_zero(rr)) return jac_dbl(p);
    return jac_infinity<F>();
  }
  F I = F_sqr(F_dbl(H));
  F J = F_mul(H, I);
  F V = F_mul(U1, I);
  jac<F> r;
  r.x = F_sub(F_sub(F_sqr(rr), J), F_dbl(V));
  r.y = F_sub(F_mul(rr, F_sub(V, r.x)), F_dbl(F_mul(S1, J)));
  r.z = F_mul(F_sub(F_sub(F_sqr(F_add(p.z, q.z)), Z1Z1), Z2Z2), H);
  return r;
}
template <class F>
BLS_INL jac<F> jac_add(const jac<F>& p, const jac<F>& q) {
  if constexpr (lazy_curve<F>::add)
    return jac_add_lazy(p, q);
  else
    return jac_add_eager(p, q);
}

// [k]P for a 64-bit k, P affine (not infinity).  Left-to-right double-and-add.
template <class F>
BLS_HDNI jac<F> jac_mul_u64(const aff<F>& P, uint64_t k) {
  jac<F> r = jac_infinity<F>();
  if (k == 0) return r;
  int top = 63;
  while (((k >> top) & 1ull) == 0) top--;
  r = jac_from_aff(P);
  for (int i = top - 1; i >= 0; i--) {
    r = jac_dbl(r);
    if ((k >> i) & 1ull) r = jac_add_aff(r, P);
  }
  return r;
}

// [|z|]P for the BLS parameter |z| = 0xd201000000010000 (wave-uniform branches), P Jacobian.
template <class F>
BLS_HDNI jac<F> jac_mul_zabs(const jac<F>& P) {
  jac<F> r = P;
  for (int i = 62; i >= 0; i--) {
    r = jac_dbl(r);
    if ((BLS_Z_ABS >> i) & 1ull) r = jac_add(r, P);
  }
  return r;
}

// The same chain with P re-read through `loadP` at each of the five additions (|z| has Hamming weight 6), so the
// doubling loop carries only the accumulator across the product calls; holding P in registers too made the
// compiler spill it around every call.  The kernels keep P in their SoA buffers (k_hash.hip, k_sig.hip).
template <class F, class LoadP>
BLS_INL jac<F> jac_mul_zabs_ld(LoadP loadP) {
  jac<F> r = loadP();
#pragma unroll 1
  for (int i = 62; i >= 0; i--) {
    r = jac_dbl(r);
    if ((BLS_Z_ABS >> i) & 1ull) r = jac_add(r, loadP());
  }
  return r;
}
// affine P (never infinity): mixed additions
template <class F, class LoadA>
BLS_INL jac<F> jac_mul_zabs_lda(LoadA loadA) {
  jac<F> r = jac_from_aff(loadA());
#pragma unroll 1
  for (int i = 62; i >= 0; i--) {
    r = jac_dbl(r);
    if ((BLS_Z_ABS >> i) & 1ull) r = jac_add_aff(r, loadA());
  }
  return r;
}

BLS_HDNI bool jac_to_aff(const g1j& p, g1a& out) {
  if (jac_is_inf(p)) return false;
  fp zi = fp_inv(p.z);
  fp zi2 = fp_sqr(zi);
  out.x = fp_mul(p.x, zi2);
  out.y = fp_mul(p.y, fp_mul(zi2, zi));
  return true;
}
BLS_HDNI bool jac_to_aff(const g2j& p, g2a& out) {
  if (jac_is_inf(p)) return false;
  fp2 zi = fp2_inv(p.z);
  fp2 zi2 = fp2_sqr(zi);
  out.x = fp2_mul(p.x, zi2);
  out.y = fp2_mul(p.y, fp2_mul(zi2, zi));
  return true;
}

// Jacobian equality (both may be infinity)
template <class F>
BLS_FN bool jac_eq(const jac<F>& p, const jac<F>& q) {
  bool pi = jac_is_inf(p), qi = jac_is_inf(q);
  if (pi || qi) return pi && qi;
  F Z1Z1 = F_sqr(p.z), Z2Z2 = F_sqr(q.z);
  if (!F_is_zero(F_sub(F_mul(p.x, Z2Z2), F_mul(q.x, Z1Z1)))) return false;
  F a = F_mul(p.y, F_mul(q.z, Z2Z2));
  F b = F_mul(q.y, F_mul(p.z, Z1Z1));
  return F_is_zero(F_sub(a, b));
}

// ---- G2 endomorphism psi and subgroup check -------------------------------------------------------
BLS_FN g2j g2_psi(const g2j& p) {
  g2j r;
  r.x = fp2_mul(fp2_conj(p.x), PSI_X);
  r.y = fp2_mul(fp2_conj(p.y), PSI_Y);
  r.z = fp2_conj(p.z);
  return r;
}
BLS_FN g2j g2_psi2(const g2j& p) {
  g2j r;
  r.x = fp2_mul(p.x, PSI2_X);
  r.y = fp2_mul(p.y, PSI2_Y);
  r.z = p.z;
  return r;
}

// The endomorphism with eigenvalue lambda = -z^2 (mod r) on both groups, for the batch scalars r = a + b lambda
// (k_common.hpp jac_mul_scalar_word, msm.hpp): G1 phi(x, y) = (beta x, y) -- the map g1_in_subgroup checks as
// -[z^2] -- and on G2 -psi^2 (psi = [z] there, so psi^2 = [z^2]).  Both act on Jacobian coordinates directly.
BLS_FN g1j endo_lambda(const g1j& p) {
  g1j r = p;
  r.x = fp_mul(p.x, G1_BETA);
  return r;
}
BLS_FN g2j endo_lambda(const g2j& p) { return jac_neg(g2_psi2(p)); }

// P in G2  <=>  psi(P) == [z]P  (z = -|z|)   (Scott, eprint 2021/1130)
BLS_HDNI bool g2_in_subgroup(const g2a& p) {
  g2j P = jac_from_aff(p);
  g2j zP = jac_neg(jac_mul_zabs(P));
  return jac_eq(g2_psi(P), zP);
}
// the same check with the affine P read through `loadA` (k_sig_decode: from its output buffer)
template <class LoadA>
BLS_INL bool g2_in_subgroup_ld(LoadA loadA) {
  const g2j zP = jac_neg(jac_mul_zabs_lda<fp2>(loadA));
  return jac_eq(g2_psi(jac_from_aff(loadA())), zP);
}

BLS_HD bool g1_on_curve(const g1a& p) {
  return fp_eq(fp_sqr(p.y), fp_add(fp_mul(fp_sqr(p.x), p.x), FP_B1));
}
BLS_HD bool g2_on_curve(const g2a& p) {
  return fp2_eq(fp2_sqr(p.y), fp2_add(fp2_mul(fp2_sqr(p.x), p.x), FP2_B2));
}

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
BLS_HD fp2 F_add(const fp2& a, const fp2& b) { return fp2_add(a, b); }
BLS_HD fp2 F_sub(const fp2& a, const fp2& b) { return fp2_sub(a, b); }
BLS_HD fp2 F_mul(const fp2& a, const fp2& b) { return fp2_mul(a, b); }
BLS_HD fp2 F_sqr(const fp2& a) { return fp2_sqr(a); }
BLS_HD fp2 F_dbl(const fp2& a) { return fp2_dbl(a); }
BLS_HD fp2 F_neg(const fp2& a) { return fp2_neg(a); }
BLS_HD bool F_is_zero(const fp2& a) { return fp2_is_zero(a); }
BLS_HD fp2 F_select(bool c, const fp2& a, const fp2& b) { return fp2_select(c, a, b); }
BLS_HD fp2 F_add_nr(const fp2& a, const fp2& b) { return fp2_add_nr(a, b); }

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

template <class F>
BLS_FN jac<F> jac_dbl(const jac<F>& p) {
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

template <class F>
BLS_HD jac<F> jac_neg(const jac<F>& p) {
  jac<F> r = p;
  r.y = F_neg(p.y);
  return r;
}

// p + q with q affine (q never infinity here)
template <class F>
BLS_INL jac<F> jac_add_aff(const jac<F>& p, const aff<F>& q) {
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

// general Jacobian addition
template <class F>
BLS_INL jac<F> jac_add(const jac<F>& p, const jac<F>& q) {
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

// Optimal-ate Miller loop and final exponentiation for BLS12-381.  Same algorithm as
// oracle/bls12_381.py `miller_loop_proj` / `final_exp` (the oracle checks it against the definitional
// affine Miller loop and the definitional (p^12-1)/r exponentiation).
#pragma once
#include "curve.hpp"

struct g2proj {
  fp2 x, y, z;
};

// Doubling step in homogeneous projective coordinates with the tangent line evaluated at P:
//   line = (E - B) + (3 X^2 xP) v + (-H yP) v w
BLS_FN void miller_dbl_step(g2proj& T, const fp& xP, const fp& yP, fp2& l0, fp2& l1, fp2& l4) {
  fp2 A = fp2_half(fp2_mul(T.x, T.y));
  fp2 B = fp2_sqr(T.y);
  fp2 C = fp2_sqr(T.z);
  // E = 3 b' C = 12 (1+u) C
  fp2 E = fp2_mul3(fp2_mul_xi(C));
  E = fp2_dbl(fp2_dbl(E));
  fp2 F = fp2_mul3(E);
  fp2 G = fp2_half(fp2_add(B, F));
  fp2 H = fp2_sub(fp2_sub(fp2_sqr(fp2_add(T.y, T.z)), B), C);
  fp2 J = fp2_sqr(T.x);
  fp2 E2 = fp2_sqr(E);
  T.x = fp2_mul(A, fp2_sub(B, F));
  T.y = fp2_sub(fp2_sqr(G), fp2_mul3(E2));
  T.z = fp2_mul(B, H);
  l0 = fp2_sub(E, B);
  l1 = fp2_mul_fp(fp2_mul3(J), xP);
  l4 = fp2_mul_fp(fp2_neg(H), yP);
}

// Mixed addition step T + Q (Q affine) with the chord line evaluated at P:
//   line = (theta x2 - lambda y2) + (-theta xP) v + (lambda yP) v w
BLS_FN void miller_add_step(g2proj& T, const g2a& Q, const fp& xP, const fp& yP, fp2& l0, fp2& l1, fp2& l4) {
  fp2 theta = fp2_sub(T.y, fp2_mul(Q.y, T.z));
  fp2 lam = fp2_sub(T.x, fp2_mul(Q.x, T.z));
  fp2 C = fp2_sqr(theta);
  fp2 D = fp2_sqr(lam);
  fp2 E = fp2_mul(lam, D);
  fp2 F = fp2_mul(T.z, C);
  fp2 G = fp2_mul(T.x, D);
  fp2 H = fp2_sub(fp2_add(E, F), fp2_dbl(G));
  fp2 X3 = fp2_mul(lam, H);
  fp2 Y3 = fp2_sub(fp2_mul(theta, fp2_sub(G, H)), fp2_mul(T.y, E));
  fp2 Z3 = fp2_mul(T.z, E);
  l0 = fp2_sub(fp2_mul(theta, Q.x), fp2_mul(lam, Q.y));
  l1 = fp2_mul_fp(fp2_neg(theta), xP);
  l4 = fp2_mul_fp(lam, yP);
  T.x = X3;
  T.y = Y3;
  T.z = Z3;
}

// ---- Two-pass Miller loop (pipeline form) -------------------------------------------------------------
// Pass 1 (k_miller_lines) walks T over the 68 steps and emits each step's line in Q-only form
// (l0, c1, c4) with l1 = c1 xP and l4 = c4 yP; pass 2 (k_miller_acc) folds the lines into f.  Splitting the
// loop removes T/Q (and the line arithmetic) from the live state of the Fp12 accumulation, which is what
// spilled to scratch in the one-pass loop (profiles/r01_pmc_traffic.json), and makes the lines depend on
// H(m) only, so sets sharing a message can share them.  Same operations as miller_loop below.
#define MILLER_STEPS 68
struct line3 {
  fp2 l0, c1, c4;
};
// step s of the flat loop is an addition step iff the previous doubling consumed a set bit of |z|
BLS_HD bool miller_step_is_add(int s) {
  int bit = 62;
  bool add_next = false;
  for (int k = 0; k < s; k++) {
    if (!add_next) {
      add_next = (BLS_Z_ABS >> bit) & 1ull;
      bit--;
    } else {
      add_next = false;
    }
  }
  return add_next;
}
#if BLS_LAZY_CURVE
// The additive glue as lazily reduced combinations (curve.hpp F_lc): 12 b' C = 12 xi C in two steps (total weight 24).
BLS_FN void miller_dbl_line(g2proj& R, line3& Ln) {
  const fp2 A = fp2_half(fp2_mul(R.x, R.y));
  const fp2 B = fp2_sqr(R.y);
  const fp2 C = fp2_sqr(R.z);
  const fp2 xC = fp2_make(fp_lc(T<1>(C.c0), T<-1>(C.c1)), fp_lc(T<1>(C.c0), T<1>(C.c1)));
  const fp2 E = F_lc(L<12>(xC));
  const fp2 G = fp2_half(F_lc(L<1>(B), L<3>(E)));
  const fp2 H = F_lc(L<1>(fp2_sqr(fp2_add_norm(R.y, R.z))), L<-1>(B), L<-1>(C));
  const fp2 J = fp2_sqr(R.x);
  const fp2 E2 = fp2_sqr(E);
  R.x = fp2_mul(A, F_lc(L<1>(B), L<-3>(E)));
  R.y = F_lc(L<1>(fp2_sqr(G)), L<-3>(E2));
  R.z = fp2_mul(B, H);
  Ln.l0 = F_lc(L<1>(E), L<-1>(B));
  Ln.c1 = F_lc(L<3>(J));
  Ln.c4 = F_lc(L<-1>(H));
}
BLS_FN void miller_add_line(g2proj& R, const g2a& Q, line3& Ln) {
  const fp2 theta = F_lc(L<1>(R.y), L<-1>(fp2_mul(Q.y, R.z)));
  const fp2 lam = F_lc(L<1>(R.x), L<-1>(fp2_mul(Q.x, R.z)));
  const fp2 C = fp2_sqr(theta);
  const fp2 D = fp2_sqr(lam);
  const fp2 E = fp2_mul(lam, D);
  const fp2 F = fp2_mul(R.z, C);
  const fp2 G = fp2_mul(R.x, D);
  const fp2 H = F_lc(L<1>(E), L<1>(F), L<-2>(G));
  const fp2 X3 = fp2_mul(lam, H);
  const fp2 Y3 = F_lc(L<1>(fp2_mul(theta, F_lc(L<1>(G), L<-1>(H)))), L<-1>(fp2_mul(R.y, E)));
  const fp2 Z3 = fp2_mul(R.z, E);
  Ln.l0 = F_lc(L<1>(fp2_mul(theta, Q.x)), L<-1>(fp2_mul(lam, Q.y)));
  Ln.c1 = F_lc(L<-1>(theta));
  Ln.c4 = lam;
  R.x = X3;
  R.y = Y3;
  R.z = Z3;
}
#else
BLS_FN void miller_dbl_line(g2proj& T, line3& L) {
  fp2 A = fp2_half(fp2_mul(T.x, T.y));
  fp2 B = fp2_sqr(T.y);
  fp2 C = fp2_sqr(T.z);
  fp2 E = fp2_mul3(fp2_mul_xi(C));
  E = fp2_dbl(fp2_dbl(E));
  fp2 F = fp2_mul3(E);
  fp2 G = fp2_half(fp2_add(B, F));
  fp2 H = fp2_sub(fp2_sub(fp2_sqr(fp2_add(T.y, T.z)), B), C);
  fp2 J = fp2_sqr(T.x);
  fp2 E2 = fp2_sqr(E);
  T.x = fp2_mul(A, fp2_sub(B, F));
  T.y = fp2_sub(fp2_sqr(G), fp2_mul3(E2));
  T.z = fp2_mul(B, H);
  L.l0 = fp2_sub(E, B);
  L.c1 = fp2_mul3(J);
  L.c4 = fp2_neg(H);
}
BLS_FN void miller_add_line(g2proj& T, const g2a& Q, line3& L) {
  fp2 theta = fp2_sub(T.y, fp2_mul(Q.y, T.z));
  fp2 lam = fp2_sub(T.x, fp2_mul(Q.x, T.z));
  fp2 C = fp2_sqr(theta);
  fp2 D = fp2_sqr(lam);
  fp2 E = fp2_mul(lam, D);
  fp2 F = fp2_mul(T.z, C);
  fp2 G = fp2_mul(T.x, D);
  fp2 H = fp2_sub(fp2_add(E, F), fp2_dbl(G));
  fp2 X3 = fp2_mul(lam, H);
  fp2 Y3 = fp2_sub(fp2_mul(theta, fp2_sub(G, H)), fp2_mul(T.y, E));
  fp2 Z3 = fp2_mul(T.z, E);
  L.l0 = fp2_sub(fp2_mul(theta, Q.x), fp2_mul(lam, Q.y));
  L.c1 = fp2_neg(theta);
  L.c4 = lam;
  T.x = X3;
  T.y = Y3;
  T.z = Z3;
}
#endif
// f <- (s doubling && s > 0 ? f^2 : f) * line(P)
BLS_FN fp12 miller_acc_step(const fp12& f, int s, bool is_add, const line3& L, const fp& xP, const fp& yP) {
  fp12 g = (!is_add && s != 0) ? fp12_sqr(f) : f;
  return fp12_mul_by_014(g, L.l0, fp2_mul_fp(L.c1, xP), fp2_mul_fp(L.c4, yP));
}

// f = conj(f_{|z|,Q}(P)).  P, Q affine and not infinity.
// The 68 steps (63 doublings, 5 additions) run as one flat loop with a single copy of each step body:
// a doubling step squares f first (except the very first), an addition step does not.
BLS_HDNI fp12 miller_loop(const g1a& P, const g2a& Q) {
  g2proj T;
  T.x = Q.x;
  T.y = Q.y;
  T.z = fp2_one();
  fp12 f = fp12_one();
  int bit = 62;
  bool add_next = false;
#pragma unroll 1
  for (int s = 0; s < 68; s++) {
    fp2 l0, l1, l4;
    if (!add_next) {
      if (s != 0) f = fp12_sqr(f);
      miller_dbl_step(T, P.x, P.y, l0, l1, l4);
      add_next = (BLS_Z_ABS >> bit) & 1ull;
      bit--;
    } else {
      miller_add_step(T, Q, P.x, P.y, l0, l1, l4);
      add_next = false;
    }
    f = fp12_mul_by_014(f, l0, l1, l4);
  }
  return fp12_conj(f);
}

// f^|z| by square-and-multiply with cyclotomic squarings (f is in the cyclotomic subgroup: only called
// after the easy part of the final exponentiation)
BLS_HDNI fp12 fp12_pow_zabs(const fp12& f) {
  fp12 r = f;
  for (int i = 62; i >= 0; i--) {
    r = fp12_cyclotomic_sqr(r);
    if ((BLS_Z_ABS >> i) & 1ull) r = fp12_mul(r, f);
  }
  return r;
}
BLS_HD fp12 fp12_pow_z(const fp12& f) { return fp12_conj(fp12_pow_zabs(f)); }

// Coarse (called) Fp12 product for the straight-line part of the final exponentiation.
BLS_BIG fp12 fp12_mul_c(const fp12& a, const fp12& b) { return fp12_mul(a, b); }

// Final exponentiation, returns e^3 (same "== 1" answer since gcd(3, r) = 1):
//   easy part (p^6 - 1)(p^2 + 1), hard part 3(p^4 - p^2 + 1)/r = (z-1)^2 (z+p)(z^2+p^2-1) + 3
BLS_HDNI fp12 final_exponentiation(const fp12& f) {
  fp12 f1 = fp12_mul_c(fp12_conj(f), fp12_inv(f));
  fp12 m = fp12_mul_c(fp12_frob2(f1), f1);
  fp12 t = fp12_mul_c(fp12_pow_z(m), fp12_conj(m));
  t = fp12_mul_c(fp12_pow_z(t), fp12_conj(t));
  t = fp12_mul_c(fp12_pow_z(t), fp12_frob1(t));
  t = fp12_mul_c(fp12_mul_c(fp12_pow_z(fp12_pow_z(t)), fp12_frob2(t)), fp12_conj(t));
  return fp12_mul_c(t, fp12_mul_c(fp12_sqr(m), m));
}

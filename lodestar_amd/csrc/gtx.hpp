// Fp6 / Fp12 on lane pairs (fp2x.hpp): every Fp2 coefficient of the tower is split over the pair, lane k holding its
// c_k -- an Fp12 value is 6 x 14 registers per lane.  The formulas are tower.hpp's lazily reduced ones (Karatsuba
// Fp6 product, complex Fp12 squaring, the sparse 014 line product) with each output coefficient ONE fp_lc of product
// outputs; a term xi * d (xi = 1 + u) mixes the pair's coefficients -- (xi d)_0 = d_0 - d_1, (xi d)_1 = d_0 + d_1 --
// so d's partner coefficient arrives by a DPP swap and enters the combination with the lane's sign.
#pragma once
#include "fp2x.hpp"

struct fp6x {
  fp2x c0, c1, c2;
};
struct fp12x {
  fp6x c0, c1;
};

// this lane's coefficient of  sum_t W_t t + WD xi d  (terms and d: normalized, values <= 2p; total weight <= 15)
template <int WD, int... W>
BLS_FN fp2x lc_xi(const fp2x& d, const lt<W, fp2x>&... t) {
  const fp p = fp_swap(d.v);
  const fp lo = fp_lc(T<W>(t.v.v)..., T<WD>(d.v), T<-WD>(p));  // lane 0: d_0 - d_1
  const fp hi = fp_lc(T<W>(t.v.v)..., T<WD>(d.v), T<WD>(p));   // lane 1: d_1 + d_0
  return fp2x{fp2x_k() ? hi : lo};
}
BLS_HD fp2x fp2x_add_norm(const fp2x& a, const fp2x& b) { return fp2x{fp_add_norm(a.v, b.v)}; }

// Karatsuba: r0 = t0 + xi (X - t1 - t2), r1 = Y - t0 - t1 + xi t2, r2 = Z - t0 - t2 + t1.  a, b: normalized, values
// <= 4p (operand sums to fp2x_mul un-normalized, fp2x_mul's contract)
BLS_FN fp6x fp6x_mul(const fp6x& a, const fp6x& b) {
  const fp2x t0 = F_mul(a.c0, b.c0);
  const fp2x t1 = F_mul(a.c1, b.c1);
  const fp2x t2 = F_mul(a.c2, b.c2);
  fp6x r;
  {
    const fp2x X = F_mul(F_add_nr(a.c1, a.c2), F_add_nr(b.c1, b.c2));
    r.c0 = lc_xi<1>(F_lc(L<1>(X), L<-1>(t1), L<-1>(t2)), L<1>(t0));
  }
  {
    const fp2x Y = F_mul(F_add_nr(a.c0, a.c1), F_add_nr(b.c0, b.c1));
    r.c1 = lc_xi<1>(t2, L<1>(Y), L<-1>(t0), L<-1>(t1));
  }
  {
    const fp2x Z = F_mul(F_add_nr(a.c0, a.c2), F_add_nr(b.c0, b.c2));
    r.c2 = F_lc(L<1>(Z), L<-1>(t0), L<-1>(t2), L<1>(t1));
  }
  return r;
}

// (a0 + a1 w)^2 = (s - t - v t) + 2 t w with t = a0 a1, s = (a0 + a1)(a0 + v a1); v t = (xi t2, t0, t1)
BLS_FN fp12x fp12x_sqr(const fp12x& a) {
  const fp6x t = fp6x_mul(a.c0, a.c1);
  fp6x u, w;
  u.c0 = fp2x_add_norm(a.c0.c0, a.c1.c0);
  u.c1 = fp2x_add_norm(a.c0.c1, a.c1.c1);
  u.c2 = fp2x_add_norm(a.c0.c2, a.c1.c2);
  w.c0 = lc_xi<1>(a.c1.c2, L<1>(a.c0.c0));
  w.c1 = fp2x_add_norm(a.c0.c1, a.c1.c0);
  w.c2 = fp2x_add_norm(a.c0.c2, a.c1.c1);
  const fp6x s = fp6x_mul(u, w);
  fp12x r;
  r.c0.c0 = lc_xi<-1>(t.c2, L<1>(s.c0), L<-1>(t.c0));
  r.c0.c1 = F_lc(L<1>(s.c1), L<-1>(t.c1), L<-1>(t.c0));
  r.c0.c2 = F_lc(L<1>(s.c2), L<-1>(t.c2), L<-1>(t.c1));
  r.c1.c0 = F_lc(L<2>(t.c0));
  r.c1.c1 = F_lc(L<2>(t.c1));
  r.c1.c2 = F_lc(L<2>(t.c2));
  return r;
}

// f * (l0 + l1 v + l4 v w) (tower.hpp fp12_mul_by_014's lazy form): A0 = f0 (l0 + l1 v), A1 = f1 (l4 v) = (xi Q1, Q2,
// Q3), S = (f0 + f1)(l0 + (l1 + l4) v); c0 = A0 + v A1, c1 = S - A0 - A1 -- 13 Fp2 products
BLS_FN fp12x fp12x_mul_by_014(const fp12x& f, const fp2x& l0, const fp2x& l1, const fp2x& l4) {
  fp6x A0;
  {
    const fp2x t0 = F_mul(f.c0.c0, l0), t1 = F_mul(f.c0.c1, l1);
    A0.c0 = lc_xi<1>(F_mul(f.c0.c2, l1), L<1>(t0));
    A0.c1 = F_lc(L<1>(F_mul(F_add_nr(f.c0.c0, f.c0.c1), F_add_nr(l0, l1))), L<-1>(t0), L<-1>(t1));
    A0.c2 = F_lc(L<1>(F_mul(f.c0.c2, l0)), L<1>(t1));
  }
  const fp2x Q1 = F_mul(f.c1.c2, l4), Q2 = F_mul(f.c1.c0, l4), Q3 = F_mul(f.c1.c1, l4);
  fp6x b;  // f0 + f1
  b.c0 = fp2x_add_norm(f.c0.c0, f.c1.c0);
  b.c1 = fp2x_add_norm(f.c0.c1, f.c1.c1);
  b.c2 = fp2x_add_norm(f.c0.c2, f.c1.c2);
  fp12x r;
  r.c0.c0 = lc_xi<1>(Q3, L<1>(A0.c0));
  r.c0.c1 = lc_xi<1>(Q1, L<1>(A0.c1));
  r.c0.c2 = F_lc(L<1>(A0.c2), L<1>(Q2));
  // S = b (l0 + m v), m = l1 + l4: R1 = b0 l0, R2 = b1 m, R3 = b2 m, R4 = (b0 + b1)(l0 + m), R5 = b2 l0;
  // S = (R1 + xi R3, R4 - R1 - R2, R5 + R2)
  const fp2x m = fp2x_add_norm(l1, l4);
  const fp2x R1 = F_mul(b.c0, l0), R2 = F_mul(b.c1, m);
  r.c1.c1 = F_lc(L<1>(F_mul(F_add_nr(b.c0, b.c1), F_add_nr(l0, m))), L<-1>(R1), L<-1>(R2), L<-1>(A0.c1), L<-1>(Q2));
  r.c1.c0 = lc_xi<1>(F_lc(L<1>(F_mul(b.c2, m)), L<-1>(Q1)), L<1>(R1), L<-1>(A0.c0));
  r.c1.c2 = F_lc(L<1>(F_mul(b.c2, l0)), L<1>(R2), L<-1>(A0.c2), L<-1>(Q3));
  return r;
}

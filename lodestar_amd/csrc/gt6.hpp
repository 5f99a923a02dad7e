// GT (Fp12) arithmetic on SIX lanes: lane k of a group (ACC6_GROUPS groups of six per wave) holds the w-basis
// coefficient f_k of f = sum_k f_k w^k (Fp12 = Fp2[w]/(w^6 - xi), xi = 1 + u; tower slots c0.c0, c1.c0, c0.c1,
// c1.c1, c0.c2, c1.c2 for k = 0..5 -- gt_wave.hpp's basis).  Every lane of a group runs ONE instruction stream (operand
// choices are lane-dependent shuffles and selects, never branches), so a wave carries ten independent Fp12 chains at
// ~1/6 of the one-lane latency:
//   g6_mul:      c_k = sum_i a_i b_{k-i} (xi where i > k): 6 Fp2 products per lane (36 in all, schoolbook);
//   g6_cyc_sqr:  Granger-Scott squaring in the cyclotomic subgroup: lane k squares its output's Fp4 pair (3 Fp2
//                squarings, each pair's shared by two lanes), then 3 X -+ 2 f_k;
//   g6_frob, g6_conj, and the final exponentiation's one Fp6 inverse on the group's lane 0 (fp6_inv).
// The chain is pairing.hpp's final_exponentiation operation for operation (returns e^3 like it and gt_wave.hpp's), the
// oracle-pinned sequence; the check kernel (k_group.hip k_group_check6) is compared job for job against the oracle.
#pragma once
#include "k_common.hpp"
#include "gt_wave.hpp"

struct G6 {
  int base;    // the group's first lane
  uint32_t k;  // this lane's coefficient
};

// xi-twisted accumulation: acc + (tw ? xi P : P), lazily reduced
BLS_INL fp2 g6_acc(const fp2& acc, const fp2& P, bool tw) {
  return fp2_make(fp_lc(T<1>(acc.c0), T<1>(P.c0), T<-1>(fp_keep(tw, P.c1))),
                  fp_lc(T<1>(acc.c1), T<1>(P.c1), T<1>(fp_keep(tw, P.c0))));
}

BLS_INL fp2 g6_conj(const fp2& f, const G6& g);
// squaring slots: nibble k of each word = lane k's operand index i / j; bit k of the masks: doubled, twisted, empty
__device__ __constant__ const uint32_t ACC6_I[4] = {0x000000u, 0x111121u, 0x224332u, 0x050403u};
__device__ __constant__ const uint32_t ACC6_J[4] = {0x543210u, 0x432155u, 0x325544u, 0x050403u};
#define ACC6_DBL(s) ((s) == 0 ? 0x3Eu : (s) == 1 ? 0x3Bu : (s) == 2 ? 0x2Fu : 0x00u)
#define ACC6_TW(s) ((s) == 0 ? 0x00u : (s) == 1 ? 0x03u : (s) == 2 ? 0x0Fu : 0x15u)
#define ACC6_NIL(s) ((s) == 3 ? 0x2Au : 0x00u)



// f^2 on six lanes (the Miller loop's squaring; f need not be cyclotomic): g_k = sum over i + j = k (mod 6) of f_i f_j
// (xi where i + j >= 6) -- 21 Fp2 products as four product slots per lane (operands from the packed tables, one doubled
// for the cross terms, the odd lanes' 4th slot empty), folded slot by slot into a lazily reduced partial sum
BLS_INL fp2 g6_sqr(const fp2& f, const G6& g) {
  const uint32_t k = g.k;
  fp2 acc;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const int i = (int)((ACC6_I[q] >> (4 * k)) & 15u), j = (int)((ACC6_J[q] >> (4 * k)) & 15u);
    const bool dbl = (ACC6_DBL(q) >> k) & 1u, nil = (ACC6_NIL(q) >> k) & 1u, tw = (ACC6_TW(q) >> k) & 1u;
    const fp2 fi = fp2_shfl(f, g.base + i), fj = fp2_shfl(f, g.base + j);
    const fp2 x = fp2_select(nil, fp2_zero(), fp2_select(dbl, fp2_add_nr(fi, fi), fi));
    const fp2 P = fp2_mul(x, fj);
    acc = q == 0 ? P : g6_acc(acc, P, tw);  // slot 0 is never twisted
  }
  return acc;
}

// f * line(P) with the Q-only line of step `o` (column m, stride nm): h_k = f_k L0 + f_{k-2} L2 + f_{k-3} L3 (xi where
// the index wraps), L2 = c1 xP, L3 = c4 yP formed one Fp product per lane (lanes 0-3) and gathered
BLS_INL fp2 g6_line_mul(const fp2& f, const uint32_t* o, uint32_t nm, uint32_t m, const fp& xP, const fp& yP,
                        const G6& g) {
  const uint32_t k = g.k, kc = k < 3 ? k : 3;  // lanes 4, 5 repeat lane 3's product, unused
  const fp comp = fp_mul(ld_fp(o, nm, m, (int)(2 + kc) * W_FP), kc < 2 ? xP : yP);
  const fp2 L0 = ld_fp2(o, nm, m, 0);
  const fp2 L2 = fp2_make(fp_shfl(comp, g.base), fp_shfl(comp, g.base + 1));
  const fp2 L3 = fp2_make(fp_shfl(comp, g.base + 2), fp_shfl(comp, g.base + 3));
  const fp2 gm2 = fp2_shfl(f, g.base + (int)((k + 4) % 6)), gm3 = fp2_shfl(f, g.base + (int)((k + 3) % 6));
  fp2 h = fp2_mul(f, L0);
  h = g6_acc(h, fp2_mul(gm2, L2), k < 2);
  h = g6_acc(h, fp2_mul(gm3, L3), k < 3);
  return h;
}

// conj(f_{|z|,Q}(P)) from Q's stored lines (column m), P = (xP, yP): pairing.hpp miller_loop on six lanes
BLS_INL fp2 g6_miller(const uint32_t* lines, uint32_t nm, uint32_t m, const fp& xP, const fp& yP, const G6& g) {
  fp2 f = g.k == 0 ? fp2_one() : fp2_zero();
  int bit = 62;
  bool add_next = false;
#pragma unroll 1
  for (int s = 0; s < MILLER_STEPS; s++) {
    if (!add_next && s != 0) f = g6_sqr(f, g);
    f = g6_line_mul(f, lines + (size_t)s * W_LINE * nm, nm, m, xP, yP, g);
    if (!add_next) {
      add_next = (BLS_Z_ABS >> bit) & 1ull;
      bit--;
    } else {
      add_next = false;
    }
  }
  return g6_conj(f, g);
}

BLS_INL fp2 g6_mul(const fp2& a, const fp2& b, const G6& g) {
  fp2 acc = fp2_zero();
#pragma unroll 1
  for (int i = 0; i < 6; i++) {
    const fp2 ai = fp2_shfl(a, g.base + i);
    const fp2 bj = fp2_shfl(b, g.base + (int)((g.k + 6 - (uint32_t)i) % 6));
    acc = g6_acc(acc, fp2_mul(ai, bj), (uint32_t)i > g.k);
  }
  return acc;
}

BLS_INL fp2 g6_conj(const fp2& f, const G6& g) { return (g.k & 1) ? fp2_neg(f) : f; }

// Granger-Scott (tower.hpp fp12_cyclotomic_sqr): output k from the pair (p, p + 3), p = 0 for k in {0, 3}, 1 for
// {2, 5}, 2 for {1, 4}; t0 = a^2, t1 = b^2, s = (a + b)^2; X = t0 + xi t1 (k even), s - t0 - t1 (k = 3, 5), xi (s - t0
// - t1) (k = 1); out = 3 X - 2 f_k (k even) / 3 X + 2 f_k (k odd)
BLS_INL fp2 g6_cyc_sqr(const fp2& f, const G6& g) {
  const uint32_t k = g.k;
  const int p = (k == 0 || k == 3) ? 0 : ((k == 2 || k == 5) ? 1 : 2);
  const fp2 a = fp2_shfl(f, g.base + p), b = fp2_shfl(f, g.base + p + 3);
  const fp2 t0 = fp2_sqr(a), t1 = fp2_sqr(b), s = fp2_sqr(fp2_add_norm(a, b));
  const fp2 X0 = fp2_make(fp_lc(T<1>(t0.c0), T<1>(t1.c0), T<-1>(t1.c1)), fp_lc(T<1>(t0.c1), T<1>(t1.c0), T<1>(t1.c1)));
  const fp2 Y = fp2_make(fp_lc(T<1>(s.c0), T<-1>(t0.c0), T<-1>(t1.c0)), fp_lc(T<1>(s.c1), T<-1>(t0.c1), T<-1>(t1.c1)));
  const fp2 Y2 = fp2_make(fp_lc(T<1>(Y.c0), T<-1>(Y.c1)), fp_lc(T<1>(Y.c0), T<1>(Y.c1)));
  const bool odd = k & 1;
  const fp2 X = fp2_select(!odd, X0, fp2_select(k == 1, Y2, Y));
  return fp2_make(fp_lc(T<3>(X.c0), T<2>(fp_keep(odd, f.c0)), T<-2>(fp_keep(!odd, f.c0))),
                  fp_lc(T<3>(X.c1), T<2>(fp_keep(odd, f.c1)), T<-2>(fp_keep(!odd, f.c1))));
}

// f^(p^e), e = 1 or 2 (tower.hpp fp12_frob1 / fp12_frob2): coefficient k -> conj^e(f_k) gamma_{e,k} (gamma_{e,0} = 1)
BLS_INL fp2 g6_frob(const fp2& f, int e, const G6& g) {
  const fp2 x = e == 1 ? fp2_conj(f) : f;
  fp2 gam = fp2_one();
#pragma unroll
  for (int kk = 1; kk < 6; kk++) gam = fp2_select(g.k == (uint32_t)kk, frob_const(e, kk), gam);
  return fp2_mul(x, gam);
}

BLS_INL fp2 g6_pow_z(const fp2& x, const G6& g) {  // x^z (z < 0: conj of x^|z|), x cyclotomic
  fp2 y = x;
#pragma unroll 1
  for (int i = 62; i >= 0; i--) {
    y = g6_cyc_sqr(y, g);
    if ((BLS_Z_ABS >> i) & 1ull) y = g6_mul(y, x, g);
  }
  return g6_conj(y, g);
}

// pairing.hpp final_exponentiation on six lanes; returns e^3
BLS_INL fp2 g6_final_exp(const fp2& f, const G6& g) {
  // f1 = conj(f) / f = conj(f)^2 / (f conj(f)), f conj(f) in Fp6 (even coefficients): lane 0 inverts it
  fp2 V = g6_conj(f, g);
  fp2 U = g6_mul(f, V, g);
  V = g6_mul(V, V, g);
  const fp2 u0 = fp2_shfl(U, g.base), u2 = fp2_shfl(U, g.base + 2), u4 = fp2_shfl(U, g.base + 4);
  fp6 inv = fp6_zero();
  if (g.k == 0) inv = fp6_inv(fp6_make(u0, u2, u4));
  const fp2 i0 = fp2_shfl(inv.c0, g.base), i1 = fp2_shfl(inv.c1, g.base), i2 = fp2_shfl(inv.c2, g.base);
  U = fp2_select(g.k & 1, fp2_zero(), fp2_select(g.k == 0, i0, fp2_select(g.k == 2, i1, i2)));
  V = g6_mul(V, U, g);  // f1
  const fp2 M = g6_mul(g6_frob(V, 2, g), V, g);  // m = f1^(p^2) f1
  fp2 Tt = g6_mul(g6_pow_z(M, g), g6_conj(M, g), g);  // m^z conj(m)
  Tt = g6_mul(g6_pow_z(Tt, g), g6_conj(Tt, g), g);   // t^z conj(t)
  Tt = g6_mul(g6_pow_z(Tt, g), g6_frob(Tt, 1, g), g);  // t^z t^p
  fp2 X = g6_pow_z(g6_pow_z(Tt, g), g);
  X = g6_mul(X, g6_frob(Tt, 2, g), g);
  Tt = g6_mul(X, g6_conj(Tt, g), g);  // t^(z^2) t^(p^2) conj(t)
  U = g6_mul(g6_mul(M, M, g), M, g);
  return g6_mul(Tt, U, g);  // t m^3
}

// every lane of the group: f == 1
BLS_INL bool g6_is_one(const fp2& f, const G6& g) {
  const int mine = fp2_eq(f, g.k == 0 ? fp2_one() : fp2_zero()) ? 1 : 0;
  int all = 1;
#pragma unroll
  for (int i = 0; i < 6; i++) all &= __shfl(mine, g.base + i);
  return all != 0;
}

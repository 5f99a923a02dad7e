// Cooperative G2 Jacobian doubling chains for the latency-bound small runs (gossip flushes, block import).
//
// A small run has a few hundred messages / signatures at most, so lane-per-point code leaves the chip idle and each
// lane runs its [|z|]-chains (cofactor clearing: 126 doublings; the subgroup check: 63) one Fp2 product after the
// other: ~21 us per doubling (tools/microbench/lat_probe.hip).  Here a GROUP of 16 lanes owns one point and a
// doubling (dbl-2009-l, the formula of curve.hpp jac_dbl) runs as three product phases of independent Fp products,
// one per lane, each feeding the next straight from the products (the squarings' components ARE products; only the
// Karatsuba products and the linear combinations need a lazily reduced recombination, lacc.hpp):
//   P1 (7 lanes)  A = X^2 (2), B = Y^2 (2), Y Z (3, Karatsuba)
//   P2 (6 lanes)  C = B^2 (2), T = (X + B)^2 (2), F = (3A)^2 (2)
//   R1 (6 lanes)  W = D - X3 = 6T - 6A - 6C - F, X3 = F - 4T + 4A + 4C, Z3 = 2 Y Z
//   P3 (3 lanes)  E W (Karatsuba, E = 3A)
//   R2 (2 lanes)  Y3 = E W - 8C
// (D = 2(T - A - C)), so a doubling costs three product latencies and two recombinations, ~3x less than the serial
// form.  The additions of a chain (five per [|z|]) run on the group's lane 0 with the register code of curve.hpp.
// The phases are plain functions of (group LDS, lane in group) so the host build (tests/native/emu.cpp) runs them
// lane by lane; g2c_sync() separates them on the device.
#pragma once
#include "curve.hpp"
#include "lacc.hpp"

#define G2C_LANES 16  // lanes per group (one point)
// Fp slots of a group's LDS area
#define G2C_R 0    // the point: x0, x1, y0, y1, z0, z1
#define G2C_S 6    // products: A0 A1 B0 B1 K0 K1 K2 | C0 C1 T0 T1 F0 F1 | P0 P1 P2
#define G2C_W 22   // W0, W1
#define G2C_FPS 24
#define G2C_WORDS (G2C_FPS * BLS_NL)

BLS_INL void g2c_st_point(uint32_t* g, const g2j& p) {
  lds_st(g, G2C_R + 0, p.x.c0);
  lds_st(g, G2C_R + 1, p.x.c1);
  lds_st(g, G2C_R + 2, p.y.c0);
  lds_st(g, G2C_R + 3, p.y.c1);
  lds_st(g, G2C_R + 4, p.z.c0);
  lds_st(g, G2C_R + 5, p.z.c1);
}
BLS_INL g2j g2c_ld_point(const uint32_t* g) {
  g2j p;
  p.x = fp2_make(lds_ld(g, G2C_R + 0), lds_ld(g, G2C_R + 1));
  p.y = fp2_make(lds_ld(g, G2C_R + 2), lds_ld(g, G2C_R + 3));
  p.z = fp2_make(lds_ld(g, G2C_R + 4), lds_ld(g, G2C_R + 5));
  return p;
}

// 3a for a normalized a <= 2p: normalized, <= 6p... values here are products (< 1.04p), so 3a < 3.2p <= 4p
BLS_INL fp g2c_mul3(const fp& a) { return fp_add_norm(fp_add_norm(a, a), a); }

BLS_INL void g2c_dbl_p1(uint32_t* g, uint32_t tg) {
  if (tg < 7) {
    fp X, Y;
    if (tg < 2)
      sqr_operands(lds_ld(g, G2C_R + 0), lds_ld(g, G2C_R + 1), (int)tg, X, Y);
    else if (tg < 4)
      sqr_operands(lds_ld(g, G2C_R + 2), lds_ld(g, G2C_R + 3), (int)tg - 2, X, Y);
    else
      kara_operands(lds_ld(g, G2C_R + 2), lds_ld(g, G2C_R + 3), lds_ld(g, G2C_R + 4), lds_ld(g, G2C_R + 5),
                    (int)tg - 4, X, Y);
    lds_st(g, G2C_S + tg, fp_mul(X, Y));
  }
}
BLS_INL void g2c_dbl_p2(uint32_t* g, uint32_t tg) {
  if (tg < 6) {
    fp x0, x1;
    if (tg < 2) {  // C = B^2
      x0 = lds_ld(g, G2C_S + 2);
      x1 = lds_ld(g, G2C_S + 3);
    } else if (tg < 4) {  // T = (X + B)^2
      x0 = fp_add_norm(lds_ld(g, G2C_R + 0), lds_ld(g, G2C_S + 2));
      x1 = fp_add_norm(lds_ld(g, G2C_R + 1), lds_ld(g, G2C_S + 3));
    } else {  // F = (3A)^2
      x0 = g2c_mul3(lds_ld(g, G2C_S + 0));
      x1 = g2c_mul3(lds_ld(g, G2C_S + 1));
    }
    fp X, Y;
    sqr_operands(x0, x1, (int)(tg & 1), X, Y);
    lds_st(g, G2C_S + 7 + tg, fp_mul(X, Y));
  }
}
// lacc of sum_j c_j S[j] over the products (coefficients -8..6)
BLS_INL void g2c_lacc_term(lacc& a, const uint32_t* g, int slot, int coef) {
  const fp v = lds_ld(g, slot);
  for (int k = 0; k < (coef < 0 ? -coef : coef); k++) {
    if (coef > 0)
      lacc_add(a, v);
    else
      lacc_sub(a, v);
  }
}
BLS_INL void g2c_dbl_r1(uint32_t* g, uint32_t tg) {
  if (tg < 6) {
    const int c = (int)(tg & 1);
    // products of component c: A_c = S[c], C_c = S[7 + c], T_c = S[9 + c], F_c = S[11 + c]
    lacc a;
    lacc_init(a);
    int dst;
    if (tg < 2) {  // W = 6T - 6A - 6C - F
      g2c_lacc_term(a, g, G2C_S + 9 + c, 6);
      g2c_lacc_term(a, g, G2C_S + c, -6);
      g2c_lacc_term(a, g, G2C_S + 7 + c, -6);
      g2c_lacc_term(a, g, G2C_S + 11 + c, -1);
      dst = G2C_W + c;
    } else if (tg < 4) {  // X3 = F - 4T + 4A + 4C
      g2c_lacc_term(a, g, G2C_S + 11 + c, 1);
      g2c_lacc_term(a, g, G2C_S + 9 + c, -4);
      g2c_lacc_term(a, g, G2C_S + c, 4);
      g2c_lacc_term(a, g, G2C_S + 7 + c, 4);
      dst = G2C_R + c;
    } else {  // Z3 = 2 Y Z: 2 (K0 - K1) + 2 (K2 - K0 - K1) u
      if (c == 0) {
        g2c_lacc_term(a, g, G2C_S + 4, 2);
        g2c_lacc_term(a, g, G2C_S + 5, -2);
      } else {
        g2c_lacc_term(a, g, G2C_S + 6, 2);
        g2c_lacc_term(a, g, G2C_S + 4, -2);
        g2c_lacc_term(a, g, G2C_S + 5, -2);
      }
      dst = G2C_R + 4 + c;
    }
    lds_st(g, dst, lacc_fin(a));
  }
}
BLS_INL void g2c_dbl_p3(uint32_t* g, uint32_t tg) {
  if (tg < 3) {
    const fp e0 = g2c_mul3(lds_ld(g, G2C_S + 0)), e1 = g2c_mul3(lds_ld(g, G2C_S + 1));
    fp X, Y;
    kara_operands(e0, e1, lds_ld(g, G2C_W + 0), lds_ld(g, G2C_W + 1), (int)tg, X, Y);
    lds_st(g, G2C_S + 13 + tg, fp_mul(X, Y));
  }
}
BLS_INL void g2c_dbl_r2(uint32_t* g, uint32_t tg) {
  if (tg < 2) {
    const int c = (int)tg;
    lacc a;
    lacc_init(a);
    if (c == 0) {  // P0 - P1 - 8 C0
      g2c_lacc_term(a, g, G2C_S + 13, 1);
      g2c_lacc_term(a, g, G2C_S + 14, -1);
    } else {  // P2 - P0 - P1 - 8 C1
      g2c_lacc_term(a, g, G2C_S + 15, 1);
      g2c_lacc_term(a, g, G2C_S + 13, -1);
      g2c_lacc_term(a, g, G2C_S + 14, -1);
    }
    g2c_lacc_term(a, g, G2C_S + 7 + c, -8);
    lds_st(g, G2C_R + 2 + c, lacc_fin(a));
  }
}

#if defined(__HIPCC__)
__device__ __forceinline__ void g2c_sync() { __syncthreads(); }
// one cooperative doubling of every group's point (all lanes of the workgroup call it)
__device__ __forceinline__ void g2c_dbl(uint32_t* g, uint32_t tg) {
  g2c_dbl_p1(g, tg);
  g2c_sync();
  g2c_dbl_p2(g, tg);
  g2c_sync();
  g2c_dbl_r1(g, tg);
  g2c_sync();
  g2c_dbl_p3(g, tg);
  g2c_sync();
  g2c_dbl_r2(g, tg);
  g2c_sync();
}
// R <- [|z|] R with the additions of P on lane 0 (loadP: P, Jacobian, read where it is needed; jac_add handles the
// exceptional cases).  Every lane of the workgroup calls it (the barriers); R in the group's LDS on entry and exit;
// a group with `on` false (no point) runs the phases on its own LDS and never calls loadP.
template <class LoadP>
__device__ void g2c_mul_zabs(uint32_t* g, uint32_t tg, bool on, LoadP loadP) {
#pragma unroll 1
  for (int i = 62; i >= 0; i--) {
    g2c_dbl(g, tg);
    if ((BLS_Z_ABS >> i) & 1ull) {
      if (tg == 0 && on) g2c_st_point(g, jac_add(g2c_ld_point(g), loadP()));
      g2c_sync();
    }
  }
}
#else
// host model of the same schedule (tests): phases lane by lane, a group of one
template <class LoadP>
static g2j g2c_host_mul_zabs(const g2j& P, LoadP loadP) {
  uint32_t g[G2C_WORDS];
  g2c_st_point(g, P);
  for (int i = 62; i >= 0; i--) {
    for (uint32_t t = 0; t < G2C_LANES; t++) g2c_dbl_p1(g, t);
    for (uint32_t t = 0; t < G2C_LANES; t++) g2c_dbl_p2(g, t);
    for (uint32_t t = 0; t < G2C_LANES; t++) g2c_dbl_r1(g, t);
    for (uint32_t t = 0; t < G2C_LANES; t++) g2c_dbl_p3(g, t);
    for (uint32_t t = 0; t < G2C_LANES; t++) g2c_dbl_r2(g, t);
    if ((BLS_Z_ABS >> i) & 1ull) g2c_st_point(g, jac_add(g2c_ld_point(g), loadP()));
  }
  return g2c_ld_point(g);
}
#endif

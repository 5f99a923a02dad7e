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
#define G2C_Q 24   // the addend of g2c_add: x0, x1, y0, y1, z0, z1; slots 30 .. 67: its products and sums
#define G2C_FPS 68
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
BLS_INL void g2c_dbl_r1(uint32_t* g, uint32_t tg) {
  if (tg < 6) {
    const int c = (int)(tg & 1);
    // products of component c: A_c = S[c], C_c = S[7 + c], T_c = S[9 + c], F_c = S[11 + c]
    lacc a;
    lacc_init(a);
    int dst;
    if (tg < 2) {  // W = 6T - 6A - 6C - F
      lacc_term(a, g, G2C_S + 9 + c, 6);
      lacc_term(a, g, G2C_S + c, -6);
      lacc_term(a, g, G2C_S + 7 + c, -6);
      lacc_term(a, g, G2C_S + 11 + c, -1);
      dst = G2C_W + c;
    } else if (tg < 4) {  // X3 = F - 4T + 4A + 4C
      lacc_term(a, g, G2C_S + 11 + c, 1);
      lacc_term(a, g, G2C_S + 9 + c, -4);
      lacc_term(a, g, G2C_S + c, 4);
      lacc_term(a, g, G2C_S + 7 + c, 4);
      dst = G2C_R + c;
    } else {  // Z3 = 2 Y Z: 2 (K0 - K1) + 2 (K2 - K0 - K1) u
      if (c == 0) {
        lacc_term(a, g, G2C_S + 4, 2);
        lacc_term(a, g, G2C_S + 5, -2);
      } else {
        lacc_term(a, g, G2C_S + 6, 2);
        lacc_term(a, g, G2C_S + 4, -2);
        lacc_term(a, g, G2C_S + 5, -2);
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
      lacc_term(a, g, G2C_S + 13, 1);
      lacc_term(a, g, G2C_S + 14, -1);
    } else {  // P2 - P0 - P1 - 8 C1
      lacc_term(a, g, G2C_S + 15, 1);
      lacc_term(a, g, G2C_S + 13, -1);
      lacc_term(a, g, G2C_S + 14, -1);
    }
    lacc_term(a, g, G2C_S + 7 + c, -8);
    lds_st(g, G2C_R + 2 + c, lacc_fin(a));
  }
}

// ---- cooperative addition R <- R + Q (Q in the G2C_Q slots; the formula of curve.hpp jac_add) -------------------
//   P1 (12 lanes)  Z1Z1 (2), Z2Z2 (2), Y1 Z2 (3), Y2 Z1 (3), (Z1 + Z2)^2 (2)              -> 30 .. 41
//   R1 (6 lanes)   Y1 Z2, Y2 Z1, ZZ = (Z1 + Z2)^2 - Z1Z1 - Z2Z2                           -> 42 .. 47
//   P2 (12 lanes)  U1 = X1 Z2Z2, U2 = X2 Z1Z1, S1 = Y1Z2 Z2Z2, S2 = Y2Z1 Z1Z1 (3 each)    -> 48 .. 59
//   R2 (8 lanes)   H = U2 - U1, r = 2 (S2 - S1), U1, S1                                    -> 60 .. 67
//   P3 (7 lanes)   I = (2H)^2 (2), r^2 (2), ZZ H (3)                                       -> 30 .. 36
//   R3 (2 lanes)   Z3 = ZZ H                                                               -> 37, 38
//   P4 (6 lanes)   J = H I, V = U1 I (3 each)                                              -> 48 .. 53
//   R4 (6 lanes)   X3 = r^2 - J - 2V, W = V - X3 = 3V - r^2 + J, J                          -> 54 .. 59
//   P5 (6 lanes)   r W, S1 J (3 each)                                                      -> 39 .. 44
//   R5 (6 lanes)   R = (X3, Y3 = r W - 2 S1 J, Z3)
// Five product latencies and five recombinations (~19 us vs ~45 us for jac_add on one lane).  The exceptional
// cases (an infinite operand, H = 0) are detected by the writer lanes of R5 from the operands, which stay in place
// until then, and lane 0 writes jac_add's result instead: every group passes the same barriers.
#define G2C_A 30
BLS_INL void g2c_add_p1(uint32_t* g, uint32_t tg) {
  if (tg < 12) {
    fp X, Y;
    if (tg < 2)
      sqr_operands(lds_ld(g, G2C_R + 4), lds_ld(g, G2C_R + 5), (int)tg, X, Y);
    else if (tg < 4)
      sqr_operands(lds_ld(g, G2C_Q + 4), lds_ld(g, G2C_Q + 5), (int)tg - 2, X, Y);
    else if (tg < 7)
      kara_operands(lds_ld(g, G2C_R + 2), lds_ld(g, G2C_R + 3), lds_ld(g, G2C_Q + 4), lds_ld(g, G2C_Q + 5),
                    (int)tg - 4, X, Y);
    else if (tg < 10)
      kara_operands(lds_ld(g, G2C_Q + 2), lds_ld(g, G2C_Q + 3), lds_ld(g, G2C_R + 4), lds_ld(g, G2C_R + 5),
                    (int)tg - 7, X, Y);
    else
      sqr_operands(fp_add_norm(lds_ld(g, G2C_R + 4), lds_ld(g, G2C_Q + 4)),
                   fp_add_norm(lds_ld(g, G2C_R + 5), lds_ld(g, G2C_Q + 5)), (int)tg - 10, X, Y);
    lds_st(g, G2C_A + tg, fp_mul(X, Y));
  }
}
BLS_INL void g2c_add_r1(uint32_t* g, uint32_t tg) {
  if (tg < 6) {
    const int c = (int)(tg & 1);
    lacc a;
    lacc_init(a);
    if (tg < 2) {
      lacc_kara(a, g, G2C_A + 4, c, 1);  // Y1 Z2
    } else if (tg < 4) {
      lacc_kara(a, g, G2C_A + 7, c, 1);  // Y2 Z1
    } else {  // (Z1 + Z2)^2 - Z1Z1 - Z2Z2 (the squares' components are products)
      lacc_term(a, g, G2C_A + 10 + c, 1);
      lacc_term(a, g, G2C_A + c, -1);
      lacc_term(a, g, G2C_A + 2 + c, -1);
    }
    lds_st(g, G2C_A + 12 + tg, lacc_fin(a));
  }
}
BLS_INL void g2c_add_p2(uint32_t* g, uint32_t tg) {
  if (tg < 12) {
    const int m = (int)tg / 3, c = (int)tg % 3;
    // (a, b): U1 = X1 Z2Z2, U2 = X2 Z1Z1, S1 = Y1Z2 Z2Z2, S2 = Y2Z1 Z1Z1
    const int a = m == 0 ? G2C_R : m == 1 ? G2C_Q : m == 2 ? G2C_A + 12 : G2C_A + 14;
    const int b = (m == 0 || m == 2) ? G2C_A + 2 : G2C_A;
    fp X, Y;
    kara_operands(lds_ld(g, a), lds_ld(g, a + 1), lds_ld(g, b), lds_ld(g, b + 1), c, X, Y);
    lds_st(g, G2C_A + 18 + tg, fp_mul(X, Y));
  }
}
BLS_INL void g2c_add_r2(uint32_t* g, uint32_t tg) {
  if (tg < 8) {
    const int c = (int)(tg & 1), k = (int)tg >> 1;
    constexpr int U1 = G2C_A + 18, U2 = G2C_A + 21, S1 = G2C_A + 24, S2 = G2C_A + 27;
    lacc a;
    lacc_init(a);
    if (k == 0) {  // H
      lacc_kara(a, g, U2, c, 1);
      lacc_kara(a, g, U1, c, -1);
    } else if (k == 1) {  // r
      lacc_kara(a, g, S2, c, 2);
      lacc_kara(a, g, S1, c, -2);
    } else {  // U1, S1
      lacc_kara(a, g, k == 2 ? U1 : S1, c, 1);
    }
    lds_st(g, G2C_A + 30 + tg, lacc_fin(a));
  }
}
#define G2C_H (G2C_A + 30)
#define G2C_RR (G2C_A + 32)
#define G2C_U1 (G2C_A + 34)
#define G2C_S1 (G2C_A + 36)
BLS_INL void g2c_add_p3(uint32_t* g, uint32_t tg) {
  if (tg < 7) {
    fp X, Y;
    if (tg < 2) {
      const fp h0 = lds_ld(g, G2C_H), h1 = lds_ld(g, G2C_H + 1);
      sqr_operands(fp_add_norm(h0, h0), fp_add_norm(h1, h1), (int)tg, X, Y);
    } else if (tg < 4) {
      sqr_operands(lds_ld(g, G2C_RR), lds_ld(g, G2C_RR + 1), (int)tg - 2, X, Y);
    } else {
      kara_operands(lds_ld(g, G2C_A + 16), lds_ld(g, G2C_A + 17), lds_ld(g, G2C_H), lds_ld(g, G2C_H + 1),
                    (int)tg - 4, X, Y);
    }
    lds_st(g, G2C_A + tg, fp_mul(X, Y));  // I 30, 31; r^2 32, 33; ZZ H 34 .. 36
  }
}
BLS_INL void g2c_add_r3(uint32_t* g, uint32_t tg) {
  if (tg < 2) {
    lacc a;
    lacc_init(a);
    lacc_kara(a, g, G2C_A + 4, (int)tg, 1);
    lds_st(g, G2C_A + 7 + tg, lacc_fin(a));  // Z3: 37, 38
  }
}
BLS_INL void g2c_add_p4(uint32_t* g, uint32_t tg) {
  if (tg < 6) {
    const int b = tg < 3 ? G2C_H : G2C_U1, c = (int)tg % 3;
    fp X, Y;
    kara_operands(lds_ld(g, b), lds_ld(g, b + 1), lds_ld(g, G2C_A), lds_ld(g, G2C_A + 1), c, X, Y);
    lds_st(g, G2C_A + 18 + tg, fp_mul(X, Y));  // J 48 .. 50, V 51 .. 53
  }
}
BLS_INL void g2c_add_r4(uint32_t* g, uint32_t tg) {
  if (tg < 6) {
    const int c = (int)(tg & 1), k = (int)tg >> 1;
    constexpr int J = G2C_A + 18, V = G2C_A + 21;
    lacc a;
    lacc_init(a);
    if (k == 0) {  // X3 = r^2 - J - 2V
      lacc_term(a, g, G2C_A + 2 + c, 1);
      lacc_kara(a, g, J, c, -1);
      lacc_kara(a, g, V, c, -2);
    } else if (k == 1) {  // W = 3V - r^2 + J
      lacc_kara(a, g, V, c, 3);
      lacc_term(a, g, G2C_A + 2 + c, -1);
      lacc_kara(a, g, J, c, 1);
    } else {  // J
      lacc_kara(a, g, J, c, 1);
    }
    lds_st(g, G2C_A + 24 + tg, lacc_fin(a));  // X3 54, 55; W 56, 57; J 58, 59
  }
}
BLS_INL void g2c_add_p5(uint32_t* g, uint32_t tg) {
  if (tg < 6) {
    const int c = (int)tg % 3;
    const int a = tg < 3 ? G2C_RR : G2C_S1, b = tg < 3 ? G2C_A + 26 : G2C_A + 28;
    fp X, Y;
    kara_operands(lds_ld(g, a), lds_ld(g, a + 1), lds_ld(g, b), lds_ld(g, b + 1), c, X, Y);
    lds_st(g, G2C_A + 9 + tg, fp_mul(X, Y));  // r W 39 .. 41, S1 J 42 .. 44
  }
}
BLS_INL bool g2c_add_exceptional(const uint32_t* g) {
  return fp2_is_zero(fp2_make(lds_ld(g, G2C_R + 4), lds_ld(g, G2C_R + 5))) ||
         fp2_is_zero(fp2_make(lds_ld(g, G2C_Q + 4), lds_ld(g, G2C_Q + 5))) ||
         fp2_is_zero(fp2_make(lds_ld(g, G2C_H), lds_ld(g, G2C_H + 1)));
}
BLS_INL g2j g2c_ld_q(const uint32_t* g) { return g2c_ld_point(g + (G2C_Q - G2C_R) * BLS_NL); }
BLS_INL void g2c_st_q(uint32_t* g, const g2j& q) { g2c_st_point(g + (G2C_Q - G2C_R) * BLS_NL, q); }
// writer lane tg < 6 of R5: reads g, writes w (the same buffer on the device: the lanes of a group share a wave
// and all read before any writes; the host model writes a copy)
// the exceptional cases' lane-serial addition, out of line: inlined, jac_add's temporaries would raise the register
// pressure of every chain loop that adds (the subgroup check's loop spilled ~200 scratch accesses)
#if defined(__HIPCC__)
__device__ __noinline__
#else
static
#endif
void g2c_add_exc(const uint32_t* g, uint32_t* w) { g2c_st_point(w, jac_add(g2c_ld_point(g), g2c_ld_q(g))); }
BLS_INL void g2c_add_r5(const uint32_t* g, uint32_t* w, uint32_t tg, bool exc) {
  if (exc) {
    if (tg == 0) g2c_add_exc(g, w);
    return;
  }
  fp v;
  if (tg < 2) {
    v = lds_ld(g, G2C_A + 24 + tg);  // X3
  } else if (tg < 4) {  // Y3 = r W - 2 S1 J
    const int c = (int)tg - 2;
    lacc a;
    lacc_init(a);
    lacc_kara(a, g, G2C_A + 9, c, 1);
    lacc_kara(a, g, G2C_A + 12, c, -2);
    v = lacc_fin(a);
  } else {
    v = lds_ld(g, G2C_A + 7 + (tg - 4));  // Z3
  }
  lds_st(w, G2C_R + tg, v);
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
// R <- R + Q (Q in the group's G2C_Q slots), all lanes of the workgroup; a group with `on` false (no point: its
// slots hold whatever they hold) skips the exceptional-case test, so it never takes lane 0's serial path
__device__ __forceinline__ void g2c_add(uint32_t* g, uint32_t tg, bool on = true) {
  g2c_add_p1(g, tg);
  g2c_sync();
  g2c_add_r1(g, tg);
  g2c_sync();
  g2c_add_p2(g, tg);
  g2c_sync();
  g2c_add_r2(g, tg);
  g2c_sync();
  g2c_add_p3(g, tg);
  g2c_sync();
  g2c_add_r3(g, tg);
  g2c_sync();
  g2c_add_p4(g, tg);
  g2c_sync();
  g2c_add_r4(g, tg);
  g2c_sync();
  g2c_add_p5(g, tg);
  g2c_sync();
  if (tg < 6) g2c_add_r5(g, g, tg, on && g2c_add_exceptional(g));
  g2c_sync();
}
// R <- [|z|] R with cooperative additions of P (loadP: P, Jacobian, read by lane 0 into the G2C_Q slots; g2c_add
// handles the exceptional cases).  Every lane of the workgroup calls it (the barriers); R in the group's LDS on entry and exit;
// a group with `on` false (no point) runs the phases on its own LDS and never calls loadP.
template <class LoadP>
__device__ __forceinline__ void g2c_mul_zabs(uint32_t* g, uint32_t tg, bool on, LoadP loadP) {
#pragma unroll 1
  for (int i = 62; i >= 0; i--) {
    g2c_dbl(g, tg);
    if ((BLS_Z_ABS >> i) & 1ull) {
      if (tg == 0 && on) g2c_st_q(g, loadP());
      g2c_sync();
      g2c_add(g, tg, on);
    }
  }
}

#else
// host model of the same schedules (tests): phases lane by lane, a group of one
static void g2c_host_add(uint32_t* g) {
  for (uint32_t t = 0; t < G2C_LANES; t++) g2c_add_p1(g, t);
  for (uint32_t t = 0; t < G2C_LANES; t++) g2c_add_r1(g, t);
  for (uint32_t t = 0; t < G2C_LANES; t++) g2c_add_p2(g, t);
  for (uint32_t t = 0; t < G2C_LANES; t++) g2c_add_r2(g, t);
  for (uint32_t t = 0; t < G2C_LANES; t++) g2c_add_p3(g, t);
  for (uint32_t t = 0; t < G2C_LANES; t++) g2c_add_r3(g, t);
  for (uint32_t t = 0; t < G2C_LANES; t++) g2c_add_p4(g, t);
  for (uint32_t t = 0; t < G2C_LANES; t++) g2c_add_r4(g, t);
  for (uint32_t t = 0; t < G2C_LANES; t++) g2c_add_p5(g, t);
  const bool exc = g2c_add_exceptional(g);
  uint32_t w[G2C_WORDS];
  for (int i = 0; i < G2C_WORDS; i++) w[i] = g[i];
  for (uint32_t t = 0; t < 6; t++) g2c_add_r5(g, w, t, exc);
  for (int i = 0; i < G2C_WORDS; i++) g[i] = w[i];
}
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
    if ((BLS_Z_ABS >> i) & 1ull) {
      g2c_st_q(g, loadP());
      g2c_host_add(g);
    }
  }
  return g2c_ld_point(g);
}
#endif

// Workgroup-cooperative GT (Fp12) arithmetic for the latency-bound tail of a batch check.
//
// The per-group tail -- one Miller loop for (-g1, S) and one final exponentiation -- is a single serial
// chain per batch group, so lane-per-group code leaves 127 of 128 lanes of its workgroup idle and runs
// ~15k Montgomery products back to back.  Here one 128-lane workgroup owns one group and every Fp12
// operation is split into its independent Fp products, one per lane, so the chain's depth drops from
// ~36-54 products per Fp12 operation to ~1 product plus a lazily reduced recombination:
//   * Fp12 values live in LDS in the w-basis (Fp12 = Fp2[w]/(w^6 - xi), xi = 1 + u): coefficient k of
//     w^k is (c0.c0, c1.c0, c0.c1, c1.c1, c0.c2, c1.c2)[k] of the tower layout, Fp index q = 2k + comp;
//   * a product phase: lane t computes one Fp product (Karatsuba components of the Fp2 pair products) into
//     the scratch S; a recombination phase: 12 lanes each form one output Fp component as a signed sum of
//     products, accumulated unreduced (lacc) and reduced once;
//   * serial leftovers (two inversions, five Miller addition steps) run on lane 0 with the register code
//     of tower.hpp / pairing.hpp.
// Same algorithm (operation for operation) as pairing.hpp's miller_loop / final_exponentiation, which the
// oracle pins; tests/test_gpu_pipeline.py compares both against oracle/bls12_381.py.
#pragma once
#include "pairing.hpp"
#include "lacc.hpp"

#define GTW_LANES 128
#define GTW_FP12 (12 * BLS_NL)

#if defined(__HIPCC__)
BLS_INL void gtw_sync() { __syncthreads(); }
#endif

// ---------------------------------------------------------------------------------------------------
// C = A * B (C may alias A or B).  SPARSE: B is a Miller line with w-coefficients 0, 2, 3 only.
// ---------------------------------------------------------------------------------------------------
template <bool SPARSE>
BLS_INL void gtw_mul_prod(const uint32_t* A, const uint32_t* B, uint32_t* S, uint32_t t) {
  constexpr uint32_t NP = SPARSE ? 54 : 108;
  if (t < NP) {
    const int pr = t / 3, c = t % 3;
    int i, j;
    if (SPARSE) {
      i = pr / 3;
      const int jj = pr % 3;
      j = jj == 0 ? 0 : jj + 1;
    } else {
      i = pr / 6;
      j = pr % 6;
    }
    fp X, Y;
    kara_operands(lds_ld(A, 2 * i), lds_ld(A, 2 * i + 1), lds_ld(B, 2 * j), lds_ld(B, 2 * j + 1), c, X, Y);
    lds_st(S, t, fp_mul(X, Y));
  }
}
template <bool SPARSE>
BLS_INL void gtw_mul_rec(uint32_t* C, const uint32_t* S, uint32_t t) {
  if (t < 12) {
    const int k = t >> 1, comp = t & 1;
    lacc acc;
    lacc_init(acc);
#pragma unroll 1
    for (int i = 0; i < 6; i++) {
      const int j = (k - i + 6) % 6;
      const bool tw = i > k;  // i + j >= 6: the product carries w^6 = xi
      int pr;
      if (SPARSE) {
        if (j == 1 || j > 3) continue;
        pr = i * 3 + (j == 0 ? 0 : j - 1);
      } else {
        pr = i * 6 + j;
      }
      const fp P0 = lds_ld(S, 3 * pr), P1 = lds_ld(S, 3 * pr + 1), P2 = lds_ld(S, 3 * pr + 2);
      // product = (P0 - P1) + (P2 - P0 - P1) u ; times xi: (2 P0 - P2) + (P2 - 2 P1) u
      if (comp == 0) {
        lacc_add(acc, P0);
        if (tw) {
          lacc_add(acc, P0);
          lacc_sub(acc, P2);
        } else {
          lacc_sub(acc, P1);
        }
      } else {
        lacc_add(acc, P2);
        lacc_sub(acc, P1);
        if (tw)
          lacc_sub(acc, P1);
        else
          lacc_sub(acc, P0);
      }
    }
    lds_st(C, t, lacc_fin(acc));
  }
}
#if defined(__HIPCC__)
// the two phases in sequence
template <bool SPARSE>
__device__ void gtw_mul(uint32_t* C, const uint32_t* A, const uint32_t* B, uint32_t* S, uint32_t t) {
  gtw_mul_prod<SPARSE>(A, B, S, t);
  gtw_sync();
  gtw_mul_rec<SPARSE>(C, S, t);
  gtw_sync();
}

// ---------------------------------------------------------------------------------------------------
// D = A^2 in the cyclotomic subgroup (Granger-Scott, as fp12_cyclotomic_sqr in tower.hpp): the w-pairs
// (k, k+3) are Fp4 elements; 9 Fp2 squarings = 18 Fp products, then 12 recombination lanes.
// ---------------------------------------------------------------------------------------------------
// PH: bit 0 = the product phase, bit 1 = the recombination phase (the latency probe times them apart)
template <int PH = 3>
__device__ void gtw_cyc_sqr(uint32_t* D, const uint32_t* A, uint32_t* S, uint32_t t) {
  if ((PH & 1) && t < 18) {
    const int p = t / 6, sq = (t % 6) >> 1, comp = t & 1;
    fp x0, x1;
    if (sq == 0) {
      x0 = lds_ld(A, 2 * p);
      x1 = lds_ld(A, 2 * p + 1);
    } else if (sq == 1) {
      x0 = lds_ld(A, 2 * p + 6);
      x1 = lds_ld(A, 2 * p + 7);
    } else {
      x0 = fp_add_norm(lds_ld(A, 2 * p), lds_ld(A, 2 * p + 6));  // <= 4p, normalized: sqr_operands' contract
      x1 = fp_add_norm(lds_ld(A, 2 * p + 1), lds_ld(A, 2 * p + 7));
    }
    fp X, Y;
    sqr_operands(x0, x1, comp, X, Y);
    lds_st(S, t, fp_mul(X, Y));
  }
  gtw_sync();
  if ((PH & 2) && t < 12) {
    // Output k, component comp: 3 X -+ 2 z with X a signed sum of the pair's six products (t0r, t0i, t1r, t1i, sr, si)
    // = S[6p .. 6p + 5].  kind 0: c0 = xi t1 + t0 = (t1r - t1i + t0r) + (t1r + t1i + t0i) u; kind 1: c1 = s - t0 - t1;
    // kind 2: xi c1 = (c1r - c1i) + (c1r + c1i) u.  The signs come from a table (bit j of POS / NEG: product j enters
    // with + / -), so the twelve lanes run ONE instruction stream: no divergent paths per kind and component.
    const int k = t >> 1, comp = t & 1;
    const int p = (k == 0 || k == 3) ? 0 : ((k == 2 || k == 5) ? 1 : 2);
    const int kind = (k == 0 || k == 2 || k == 4) ? 0 : (k == 1 ? 2 : 1);
    // sign masks over j = t0r, t0i, t1r, t1i, sr, si: 6 bits per entry e = 2 kind + comp
    const int e = 2 * kind + comp;
    const uint32_t pos = (uint32_t)(0xc1a810385ull >> (6 * e)) & 63u, neg = (uint32_t)(0x3e5285008ull >> (6 * e)) & 63u;
    uint32_t ps[BLS_NL], ng[BLS_NL];
#pragma unroll
    for (int i = 0; i < BLS_NL; i++) ps[i] = ng[i] = 0;
#pragma unroll
    for (int j = 0; j < 6; j++) {
      const uint32_t mp = 0u - ((pos >> j) & 1u), mn = 0u - ((neg >> j) & 1u);
      const uint32_t* src = S + (6 * p + j) * BLS_NL;
#pragma unroll
      for (int i = 0; i < BLS_NL; i++) {
        const uint32_t v = src[i];
        ps[i] += v & mp;
        ng[i] += v & mn;
      }
    }
    // 3 X -+ 2 z: at most 3 products per side times 3, plus 2 z: <= 11 terms of < 2^28 per limb
    const uint32_t* zs = A + t * BLS_NL;
    const uint32_t mz = (k & 1) ? ~0u : 0u;
    lacc acc;
#pragma unroll
    for (int i = 0; i < BLS_NL; i++) {
      const uint32_t z2 = zs[i] << 1;
      acc.pos[i] = 3 * ps[i] + (z2 & mz);
      acc.neg[i] = 3 * ng[i] + (z2 & ~mz);
    }
    lds_st(D, t, lacc_fin(acc));
  }
  gtw_sync();
}

// elementwise: D = conj(A) (negate the odd w-coefficients) or a copy
__device__ void gtw_conj(uint32_t* D, const uint32_t* A, uint32_t t, bool negate_odd = true) {
  if (t < 12) {
    const fp a = lds_ld(A, t);
    lds_st(D, t, (negate_odd && ((t >> 1) & 1)) ? fp_neg(a) : a);
  }
  gtw_sync();
}
__device__ void gtw_copy(uint32_t* D, const uint32_t* A, uint32_t t) { gtw_conj(D, A, t, false); }

BLS_INL fp2 frob_const(int e, int k) {
  if (e == 1) {
    switch (k) {
      case 1: return FROB1_1;
      case 2: return FROB1_2;
      case 3: return FROB1_3;
      case 4: return FROB1_4;
      default: return FROB1_5;
    }
  }
  switch (k) {
    case 1: return FROB2_1;
    case 2: return FROB2_2;
    case 3: return FROB2_3;
    case 4: return FROB2_4;
    default: return FROB2_5;
  }
}
// D = A^(p^e), e = 1 or 2 (as fp12_frob1 / fp12_frob2): coefficient k -> conj^e(a_k) * gamma_{e,k}
__device__ void gtw_frob(uint32_t* D, const uint32_t* A, int e, uint32_t t) {
  if (t < 12) {
    const int k = t >> 1, comp = t & 1;
    fp a0 = lds_ld(A, 2 * k), a1 = lds_ld(A, 2 * k + 1);
    if (e == 1) a1 = fp_neg(a1);
    fp r;
    if (k == 0) {
      r = comp ? a1 : a0;
    } else {
      const fp2 g = frob_const(e, k);
      // re = a0 g0 - a1 g1 ; im = a0 g1 + a1 g0
      const fp u = fp_mul(a0, comp ? g.c1 : g.c0);
      const fp v = fp_mul(a1, comp ? g.c0 : g.c1);
      r = comp ? fp_add(u, v) : fp_sub(u, v);
    }
    lds_st(D, t, r);
  }
  gtw_sync();
}

// ---------------------------------------------------------------------------------------------------
// LDS <-> registers (lane-0 serial parts)
// ---------------------------------------------------------------------------------------------------
BLS_INL fp2* fp12_slot(fp12& f, int k) {
  switch (k) {
    case 0: return &f.c0.c0;
    case 1: return &f.c1.c0;
    case 2: return &f.c0.c1;
    case 3: return &f.c1.c1;
    case 4: return &f.c0.c2;
    default: return &f.c1.c2;
  }
}
__device__ __forceinline__ fp12 gtw_to_reg(const uint32_t* A) {
  fp12 f;
#pragma unroll
  for (int k = 0; k < 6; k++) *fp12_slot(f, k) = fp2_make(lds_ld(A, 2 * k), lds_ld(A, 2 * k + 1));
  return f;
}
__device__ __forceinline__ void gtw_from_reg(uint32_t* A, fp12 f) {
#pragma unroll
  for (int k = 0; k < 6; k++) {
    lds_st(A, 2 * k, fp12_slot(f, k)->c0);
    lds_st(A, 2 * k + 1, fp12_slot(f, k)->c1);
  }
}
__device__ void gtw_set_one(uint32_t* A, uint32_t t) {
  if (t < 12) lds_st(A, t, t == 0 ? FP_ONE : fp_zero());
  gtw_sync();
}

// ---------------------------------------------------------------------------------------------------
// Final exponentiation (same chain as pairing.hpp final_exponentiation; returns e^3).  F is consumed.
// Work buffers: 5 Fp12 in W (W + GTW_FP12 * i).
// ---------------------------------------------------------------------------------------------------
__device__ void gtw_pow_z(uint32_t* Y, const uint32_t* X, uint32_t* S, uint32_t t) {
  gtw_copy(Y, X, t);
#pragma unroll 1
  for (int i = 62; i >= 0; i--) {
    gtw_cyc_sqr(Y, Y, S, t);
    if ((BLS_Z_ABS >> i) & 1ull) gtw_mul<false>(Y, Y, X, S, t);
  }
  gtw_conj(Y, Y, t);  // z < 0
}

__device__ __forceinline__ void gtw_final_exp(uint32_t* F, uint32_t* W, uint32_t* S, uint32_t t) {
  uint32_t *U = W, *V = W + GTW_FP12, *M = W + 2 * GTW_FP12, *T = W + 3 * GTW_FP12, *X = W + 4 * GTW_FP12;
  // f1 = conj(f) / f = conj(f)^2 / (f conj(f)), where f conj(f) = a0^2 - v a1^2 lies in Fp6: the two Fp12
  // products are cooperative and lane 0 inverts only an Fp6 (the lane-0 Fp12 inverse took 271 us in the probe)
  gtw_conj(V, F, t);
  gtw_mul<false>(U, F, V, S, t);  // f conj(f): odd w-coefficients 0
  gtw_mul<false>(V, V, V, S, t);  // conj(f)^2
  if (t == 0) {
    const fp12 n = gtw_to_reg(U);
    gtw_from_reg(U, fp12_make(fp6_inv(n.c0), fp6_zero()));
  }
  gtw_sync();
  gtw_mul<false>(V, V, U, S, t);  // f1
  gtw_frob(U, V, 2, t);
  gtw_mul<false>(M, U, V, S, t);  // m = f1^(p^2) f1
  gtw_pow_z(U, M, S, t);
  gtw_conj(V, M, t);
  gtw_mul<false>(T, U, V, S, t);  // t = m^z conj(m)
  gtw_pow_z(U, T, S, t);
  gtw_conj(V, T, t);
  gtw_mul<false>(T, U, V, S, t);  // t = t^z conj(t)
  gtw_pow_z(U, T, S, t);
  gtw_frob(V, T, 1, t);
  gtw_mul<false>(T, U, V, S, t);  // t = t^z t^p
  gtw_pow_z(U, T, S, t);
  gtw_pow_z(X, U, S, t);
  gtw_frob(V, T, 2, t);
  gtw_mul<false>(X, X, V, S, t);
  gtw_conj(V, T, t);
  gtw_mul<false>(T, X, V, S, t);  // t = t^(z^2) t^(p^2) conj(t)
  gtw_mul<false>(U, M, M, S, t);
  gtw_mul<false>(U, U, M, S, t);
  gtw_mul<false>(F, T, U, S, t);  // t m^3
}

#endif  // __HIPCC__

// ---------------------------------------------------------------------------------------------------
// Miller loop f = conj(f_{|z|,Q}(P)) into F (as pairing.hpp miller_loop).  Q affine in LDS (QA: 4 Fp:
// x.re, x.im, y.re, y.im), P = (xP, yP) uniform.  TB: T (6 Fp), then the doubling-step temporaries
// (14 Fp).  L0 / L1: Fp12-layout line buffers (w-coefficients 0, 2, 3 used), S2: the T chain's products.
//
// Three waves (GTW_MILLER_LANES): waves 1-2 update f (square: 108 products + recombination; times the sparse
// line: 54 + recombination) while wave 0 runs the T chain that produces the lines (cooperative doubling and
// addition steps: products, linear combinations, ...), up to two lines ahead (gtw_miller_schedule).  The line
// chain depends only on T, so it leaves the critical path of the f chain (divergent lanes of ONE wave would run both
// paths in turn, hence a wave of its own).  The T chain's Fp products are all fp_mul: fp2_mul's per-lane LDS argument
// slot (tower.hpp) covers lanes 0 .. 127 only.
// ---------------------------------------------------------------------------------------------------
#define GTW_MILLER_LANES (GTW_LANES + 64)

// doubling step phases (lane t of the T-chain wave, products in S)
BLS_INL void gtw_dbl_p1(const uint32_t* TB, uint32_t* S, uint32_t t) {
  // phase 1: x y (Karatsuba, 3), y^2 (2), z^2 (2), (y + z)^2 (2), x^2 (2)
  if (t < 11) {
    const fp x0 = lds_ld(TB, 0), x1 = lds_ld(TB, 1), y0 = lds_ld(TB, 2), y1 = lds_ld(TB, 3);
    const fp z0 = lds_ld(TB, 4), z1 = lds_ld(TB, 5);
    fp X, Y;
    if (t < 3) {
      kara_operands(x0, x1, y0, y1, t, X, Y);
    } else if (t < 5) {
      sqr_operands(y0, y1, t - 3, X, Y);
    } else if (t < 7) {
      sqr_operands(z0, z1, t - 5, X, Y);
    } else if (t < 9) {
      sqr_operands(fp_add(y0, z0), fp_add(y1, z1), t - 7, X, Y);
    } else {
      sqr_operands(x0, x1, t - 9, X, Y);
    }
    lds_st(S, t, fp_mul(X, Y));
  }
}
BLS_INL void gtw_dbl_p2(uint32_t* TB, uint32_t* L, const uint32_t* S, uint32_t t) {
  uint32_t* D = TB + 6 * BLS_NL;
  // phase 2 (component lanes): A = xy/2, E = 12 xi C, F = 3E, G = (B + F)/2, H = (y+z)^2 - B - C, 3J,
  // B - F, l0 = E - B.  D slots (Fp2): 0 A, 1 B-F, 2 G, 3 E, 4 B, 5 H, 6 3J
  if (t < 2) {
    const int c = t;
    const fp P0 = lds_ld(S, 0), P1 = lds_ld(S, 1), P2 = lds_ld(S, 2);
    const fp Axy = c ? fp_sub(fp_sub(P2, P0), P1) : fp_sub(P0, P1);
    const fp B = lds_ld(S, 3 + c);
    const fp C0 = lds_ld(S, 5), C1 = lds_ld(S, 6);
    const fp xiC = c ? fp_add(C0, C1) : fp_sub(C0, C1);
    const fp E = fp_mul4(fp_mul3(xiC));
    const fp F = fp_mul3(E);
    const fp G = fp_half(fp_add(B, F));
    const fp H = fp_sub(fp_sub(lds_ld(S, 7 + c), B), lds_ld(S, 5 + c));
    lds_st(D, 0 + c, fp_half(Axy));
    lds_st(D, 2 + c, fp_sub(B, F));
    lds_st(D, 4 + c, G);
    lds_st(D, 6 + c, E);
    lds_st(D, 8 + c, B);
    lds_st(D, 10 + c, H);
    lds_st(D, 12 + c, fp_mul3(lds_ld(S, 9 + c)));
    lds_st(L, 0 + c, fp_sub(E, B));  // l0 at w^0
  }
}
BLS_INL void gtw_dbl_p3(const uint32_t* TB, uint32_t* S, const fp& xP, const fp& yP, uint32_t t) {
  const uint32_t* D = TB + 6 * BLS_NL;
  // phase 3: A (B - F) (3), G^2 (2), E^2 (2), B H (3), 3J xP (2), H yP (2)
  if (t < 14) {
    fp X, Y;
    if (t < 3) {
      kara_operands(lds_ld(D, 0), lds_ld(D, 1), lds_ld(D, 2), lds_ld(D, 3), t, X, Y);
    } else if (t < 5) {
      sqr_operands(lds_ld(D, 4), lds_ld(D, 5), t - 3, X, Y);
    } else if (t < 7) {
      sqr_operands(lds_ld(D, 6), lds_ld(D, 7), t - 5, X, Y);
    } else if (t < 10) {
      kara_operands(lds_ld(D, 8), lds_ld(D, 9), lds_ld(D, 10), lds_ld(D, 11), t - 7, X, Y);
    } else if (t < 12) {
      X = lds_ld(D, 12 + (t - 10));
      Y = xP;
    } else {
      X = lds_ld(D, 10 + (t - 12));
      Y = yP;
    }
    lds_st(S, t, fp_mul(X, Y));
  }
}
BLS_INL void gtw_dbl_p4(uint32_t* TB, uint32_t* L, const uint32_t* S, uint32_t t) {
  // phase 4: T = (A(B-F), G^2 - 3E^2, B H), l1 = 3J xP at w^2, l4 = -H yP at w^3
  if (t < 2) {
    const int c = t;
    const fp P0 = lds_ld(S, 0), P1 = lds_ld(S, 1), P2 = lds_ld(S, 2);
    lds_st(TB, 0 + c, c ? fp_sub(fp_sub(P2, P0), P1) : fp_sub(P0, P1));
    lds_st(TB, 2 + c, fp_sub(lds_ld(S, 3 + c), fp_mul3(lds_ld(S, 5 + c))));
    const fp Q0 = lds_ld(S, 7), Q1 = lds_ld(S, 8), Q2 = lds_ld(S, 9);
    lds_st(TB, 4 + c, c ? fp_sub(fp_sub(Q2, Q0), Q1) : fp_sub(Q0, Q1));
    lds_st(L, 4 + c, lds_ld(S, 10 + c));
    lds_st(L, 6 + c, fp_neg(lds_ld(S, 12 + c)));
  }
}

// addition step phases (mixed addition T + Q with the chord line; the formulas of pairing.hpp miller_add_step), lane
// t of the T-chain wave; products in S (28 slots), sums in D = TB + 6 (theta 0-1, lambda 2-3, E 4-5, H 6-7, G - H 8-9)
BLS_INL void gtw_add_q1(const uint32_t* TB, const uint32_t* QA, uint32_t* S, uint32_t t) {  // Qy Tz, Qx Tz
  if (t < 6) {
    const int q = t < 3 ? 2 : 0, c = (int)t % 3;
    fp X, Y;
    kara_operands(lds_ld(QA, q), lds_ld(QA, q + 1), lds_ld(TB, 4), lds_ld(TB, 5), c, X, Y);
    lds_st(S, (int)t, fp_mul(X, Y));
  }
}
BLS_INL void gtw_add_r1(uint32_t* TB, const uint32_t* S, uint32_t t) {  // theta = Ty - Qy Tz, lambda = Tx - Qx Tz
  if (t < 4) {
    const int k = (int)t >> 1, c = (int)t & 1;
    lacc a;
    lacc_init(a);
    lacc_term(a, TB, k ? c : 2 + c, 1);
    lacc_kara(a, S, k ? 3 : 0, c, -1);
    lds_st(TB + 6 * BLS_NL, (int)t, lacc_fin(a));
  }
}
BLS_INL void gtw_add_q2(const uint32_t* TB, const uint32_t* QA, uint32_t* S, const fp& xP, const fp& yP, uint32_t t) {
  const uint32_t* D = TB + 6 * BLS_NL;
  if (t < 14) {  // C = theta^2 (2), D = lambda^2 (2), theta Qx (3), lambda Qy (3), theta xP (2), lambda yP (2)
    fp X, Y;
    if (t < 4) {
      const int k = t < 2 ? 0 : 2;
      sqr_operands(lds_ld(D, k), lds_ld(D, k + 1), (int)t & 1, X, Y);
    } else if (t < 10) {
      const int k = t < 7 ? 0 : 2, q = t < 7 ? 0 : 2, c = t < 7 ? (int)t - 4 : (int)t - 7;
      kara_operands(lds_ld(D, k), lds_ld(D, k + 1), lds_ld(QA, q), lds_ld(QA, q + 1), c, X, Y);
    } else {
      X = lds_ld(D, t < 12 ? (int)t - 10 : 2 + (int)t - 12);
      Y = t < 12 ? xP : yP;
    }
    lds_st(S, (int)t, fp_mul(X, Y));
  }
}
BLS_INL void gtw_add_r2(const uint32_t* S, uint32_t* L, uint32_t t) {  // the line: l0, l1 = -theta xP, l4 = lambda yP
  if (t < 6) {
    const int c = (int)t & 1;
    if (t < 2) {
      lacc a;
      lacc_init(a);
      lacc_kara(a, S, 4, c, 1);
      lacc_kara(a, S, 7, c, -1);
      lds_st(L, c, lacc_fin(a));
    } else if (t < 4) {
      lds_st(L, 4 + c, fp_neg(lds_ld(S, 10 + c)));
    } else {
      lds_st(L, 6 + c, lds_ld(S, 12 + c));
    }
  }
}
BLS_INL void gtw_add_q3(const uint32_t* TB, uint32_t* S, uint32_t t) {  // E = lambda D, F = Tz C, G = Tx D
  const uint32_t* D = TB + 6 * BLS_NL;
  if (t < 9) {
    const int m = (int)t / 3, c = (int)t % 3;
    fp a0, a1;
    if (m == 0) {
      a0 = lds_ld(D, 2);
      a1 = lds_ld(D, 3);
    } else {
      a0 = lds_ld(TB, m == 1 ? 4 : 0);
      a1 = lds_ld(TB, m == 1 ? 5 : 1);
    }
    const int b = m == 1 ? 0 : 2;  // C = S0, S1; D = S2, S3 (squares: the products are the components)
    fp X, Y;
    kara_operands(a0, a1, lds_ld(S, b), lds_ld(S, b + 1), c, X, Y);
    lds_st(S, 14 + (int)t, fp_mul(X, Y));
  }
}
BLS_INL void gtw_add_r3(uint32_t* TB, const uint32_t* S, uint32_t t) {  // E, H = E + F - 2G, G - H = 3G - E - F
  if (t < 6) {
    const int k = (int)t >> 1, c = (int)t & 1;
    lacc a;
    lacc_init(a);
    if (k == 0) {
      lacc_kara(a, S, 14, c, 1);
    } else if (k == 1) {
      lacc_kara(a, S, 14, c, 1);
      lacc_kara(a, S, 17, c, 1);
      lacc_kara(a, S, 20, c, -2);
    } else {
      lacc_kara(a, S, 20, c, 3);
      lacc_kara(a, S, 14, c, -1);
      lacc_kara(a, S, 17, c, -1);
    }
    lds_st(TB + 6 * BLS_NL, 4 + (int)t, lacc_fin(a));
  }
}
BLS_INL void gtw_add_q4(const uint32_t* TB, uint32_t* S, uint32_t t) {  // lambda H, theta (G - H), Ty E, Tz E
  const uint32_t* D = TB + 6 * BLS_NL;
  if (t < 12) {
    const int m = (int)t / 3, c = (int)t % 3;
    const uint32_t* ab = m < 2 ? D : TB;
    const int ka = m == 0 ? 2 : m == 1 ? 0 : m == 2 ? 2 : 4;
    const int kb = m == 0 ? 6 : m == 1 ? 8 : 4;
    fp X, Y;
    kara_operands(lds_ld(ab, ka), lds_ld(ab, ka + 1), lds_ld(D, kb), lds_ld(D, kb + 1), c, X, Y);
    lds_st(S, (int)t, fp_mul(X, Y));
  }
}
BLS_INL void gtw_add_r4(uint32_t* TB, const uint32_t* S, uint32_t t) {  // T = (lambda H, theta (G - H) - Ty E, Tz E)
  if (t < 6) {
    const int k = (int)t >> 1, c = (int)t & 1;
    lacc a;
    lacc_init(a);
    if (k == 1) {
      lacc_kara(a, S, 3, c, 1);
      lacc_kara(a, S, 6, c, -1);
    } else {
      lacc_kara(a, S, k == 0 ? 0 : 9, c, 1);
    }
    lds_st(TB, (int)t, lacc_fin(a));
  }
}

// The loop as a schedule of phases: run(f) executes phase f for every lane of the workgroup (on the device: the
// calling lane, then a barrier; in the host model, tests/native/emu.cpp: lanes 0 .. GTW_MILLER_LANES - 1 in turn --
// within a phase no lane reads what another writes).
//
// The T chain (wave 0) and the f chain (waves 1-2) are two programs stepped once per phase:
//   T, per step: a doubling in 4 phases (products, sums, products, sums) or an addition in 8 (gtw_add_q1 .. r4);
//      its line is complete after the step's 4th phase; it starts step t only when the f chain has consumed line
//      t - 2 (two line buffers, L[t & 1]);
//   f, per step: square (products, recombination; not at step 0 or after an addition step) then times the sparse
//      line (products, recombination); the line products wait, idle, until the T chain has completed that line.
// The f chain runs 4 phases per doubling step and 2 per addition step, the T chain 4 and 8: the T chain, ahead by
// up to two lines, absorbs the five additions' extra phases instead of stalling the f chain for lane-serial ones.
template <class Run>
BLS_INL void gtw_miller_schedule(Run&& run, uint32_t* F, const uint32_t* QA, const fp& xP, const fp& yP, uint32_t* TB,
                                 uint32_t* L0, uint32_t* L1, uint32_t* S, uint32_t* S2) {
  constexpr uint32_t TW = 64;  // lanes < TW: the T-chain wave; lane TW + i: f-lane i
  constexpr int NSTEPS = 68;
  // step kinds: step 0 doubles for bit 62; after the doubling for bit b an addition if bit b of |z| is set
  uint64_t add_lo = 0, add_hi = 0;  // bit s: step s is an addition
  {
    int st = 0;
    for (int bit = 62; bit >= 0; bit--) {
      st++;  // the doubling
      if ((BLS_Z_ABS >> bit) & 1ull) {
        if (st < 64)
          add_lo |= 1ull << st;
        else
          add_hi |= 1ull << (st - 64);
        st++;
      }
    }
  }
  auto is_add = [&](int st) { return st < 64 ? ((add_lo >> st) & 1ull) != 0 : ((add_hi >> (st - 64)) & 1ull) != 0; };
  run([&](uint32_t t) {
    if (t < 6) lds_st(TB, (int)t, t < 4 ? lds_ld(QA, (int)t) : (t == 4 ? FP_ONE : fp_zero()));
    if (t < 12) lds_st(F, (int)t, t == 0 ? FP_ONE : fp_zero());
  });
  int ts = 0, tp = 0;  // T chain: step, phase within it
  int fs = 0, fp_ = 0;  // f chain: step, phase within it
  int lines_done = 0, lines_used = 0;
#pragma unroll 1
  while (fs < NSTEPS) {
    // T: may start step ts once line ts - 2 has been consumed
    const bool t_on = ts < NSTEPS && (tp > 0 || ts < lines_used + 2);
    const bool t_add = ts < NSTEPS && is_add(ts);
    uint32_t* tl = (ts & 1) ? L1 : L0;
    // f: the phases of step fs (a doubling step after step 0: 4, else 2; the first two square f)
    const bool f_sq_step = fs > 0 && !is_add(fs);
    const int f_ph = f_sq_step ? fp_ : fp_ + 2;  // 0 square products, 1 square sums, 2 line products, 3 line sums
    const bool f_on = f_ph != 2 || lines_done > fs;
    const uint32_t* fl = (fs & 1) ? L1 : L0;
    const int tpc = tp;
    run([&](uint32_t t) {
      if (t < TW) {
        if (!t_on) return;
        if (!t_add) {
          if (tpc == 0)
            gtw_dbl_p1(TB, S2, t);
          else if (tpc == 1)
            gtw_dbl_p2(TB, tl, S2, t);
          else if (tpc == 2)
            gtw_dbl_p3(TB, S2, xP, yP, t);
          else
            gtw_dbl_p4(TB, tl, S2, t);
        } else {
          switch (tpc) {
            case 0: gtw_add_q1(TB, QA, S2, t); break;
            case 1: gtw_add_r1(TB, S2, t); break;
            case 2: gtw_add_q2(TB, QA, S2, xP, yP, t); break;
            case 3: gtw_add_r2(S2, tl, t); break;
            case 4: gtw_add_q3(TB, S2, t); break;
            case 5: gtw_add_r3(TB, S2, t); break;
            case 6: gtw_add_q4(TB, S2, t); break;
            default: gtw_add_r4(TB, S2, t); break;
          }
        }
      } else if (f_on) {
        const uint32_t u = t - TW;
        if (f_ph == 0)
          gtw_mul_prod<false>(F, F, S, u);
        else if (f_ph == 1)
          gtw_mul_rec<false>(F, S, u);
        else if (f_ph == 2)
          gtw_mul_prod<true>(F, fl, S, u);
        else
          gtw_mul_rec<true>(F, S, u);
      }
    });
    if (t_on) {
      if (tp == 3) lines_done = ts + 1;
      if (++tp == (t_add ? 8 : 4)) {
        ts++;
        tp = 0;
      }
    }
    if (f_on) {
      if (f_ph == 2) lines_used = fs + 1;
      if (f_ph == 3) {
        fs++;
        fp_ = 0;
      } else {
        fp_++;
      }
    }
  }
  run([&](uint32_t t) {  // f = conj(f): negate the odd w-coefficients
    if (t < 12 && ((t >> 1) & 1)) lds_st(F, (int)t, fp_neg(lds_ld(F, (int)t)));
  });
}

#if defined(__HIPCC__)
__device__ __forceinline__ void gtw_miller_loop(uint32_t* F, const uint32_t* QA, const fp& xP, const fp& yP,
                                                uint32_t* TB, uint32_t* L0, uint32_t* L1, uint32_t* S, uint32_t* S2,
                                                uint32_t t) {
  gtw_miller_schedule(
      [&](auto&& phase) {
        phase(t);
        gtw_sync();
      },
      F, QA, xP, yP, TB, L0, L1, S, S2);
}

// Fp12 word w of the SoA tower layout in HBM (Fp2 slots c0.c0, c0.c1, c0.c2, c1.c0, c1.c1, c1.c2, W_FP words per
// Fp) -> its word in the LDS w-basis layout of this engine
__device__ __forceinline__ uint32_t gtw_lds_word(uint32_t w) {
  const uint32_t slot = w / (2 * BLS_NL), rest = w % (2 * BLS_NL);
  const uint32_t k = slot < 3 ? 2 * slot : 2 * (slot - 3) + 1;
  return k * 2 * BLS_NL + rest;
}
#endif  // __HIPCC__

// LDS footprint of one cooperative group check (words)
struct GtwLds {
  uint32_t S[108 * BLS_NL];     // per-lane products
  uint32_t F[GTW_FP12];         // accumulator
  uint32_t G[GTW_FP12];         // Miller value
  uint32_t W[5 * GTW_FP12];     // final-exponentiation temporaries
  uint32_t L[GTW_FP12];         // lines (two buffers)
  uint32_t L1[GTW_FP12];
  uint32_t S2[28 * BLS_NL];     // the Miller loop's T-chain products
  uint32_t TB[(6 + 14) * BLS_NL];  // T + doubling temporaries
  uint32_t QA[4 * BLS_NL];      // Q affine
  uint32_t flag;
};

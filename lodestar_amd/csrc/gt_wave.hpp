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
__device__ fp12 gtw_to_reg(const uint32_t* A) {
  fp12 f;
#pragma unroll
  for (int k = 0; k < 6; k++) *fp12_slot(f, k) = fp2_make(lds_ld(A, 2 * k), lds_ld(A, 2 * k + 1));
  return f;
}
__device__ void gtw_from_reg(uint32_t* A, fp12 f) {
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

__device__ void gtw_final_exp(uint32_t* F, uint32_t* W, uint32_t* S, uint32_t t) {
  uint32_t *U = W, *V = W + GTW_FP12, *M = W + 2 * GTW_FP12, *T = W + 3 * GTW_FP12, *X = W + 4 * GTW_FP12;
  if (t == 0) gtw_from_reg(U, fp12_inv(gtw_to_reg(F)));
  gtw_sync();
  gtw_conj(V, F, t);
  gtw_mul<false>(V, V, U, S, t);  // f1 = conj(f) / f
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
// line: 54 + recombination -- four barrier-separated phases per step) while wave 0 computes the NEXT step's line
// from T in the same four phases (doubling: products, linear combination, products, linear combination; addition:
// lane-serial in the first phase, on lane 0: its Fp2 products use fp2_mul's per-lane LDS slot, tower.hpp, which
// covers lanes 0 .. 127 only -- the f lanes use none).  The line chain depends only on T, so it leaves the critical path of the f
// chain; the line of step s sits in L[s & 1].  Divergent lanes of ONE wave would run both paths in turn, hence a
// wave of its own.
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

BLS_INL void gtw_add_step_lane(uint32_t* TB, const uint32_t* QA, uint32_t* L, const fp& xP, const fp& yP,
                               uint32_t t) {
  if (t == 0) {
    g2proj T;
    T.x = fp2_make(lds_ld(TB, 0), lds_ld(TB, 1));
    T.y = fp2_make(lds_ld(TB, 2), lds_ld(TB, 3));
    T.z = fp2_make(lds_ld(TB, 4), lds_ld(TB, 5));
    g2a Q;
    Q.x = fp2_make(lds_ld(QA, 0), lds_ld(QA, 1));
    Q.y = fp2_make(lds_ld(QA, 2), lds_ld(QA, 3));
    fp2 l0, l1, l4;
    miller_add_step(T, Q, xP, yP, l0, l1, l4);
    lds_st(TB, 0, T.x.c0);
    lds_st(TB, 1, T.x.c1);
    lds_st(TB, 2, T.y.c0);
    lds_st(TB, 3, T.y.c1);
    lds_st(TB, 4, T.z.c0);
    lds_st(TB, 5, T.z.c1);
    lds_st(L, 0, l0.c0);
    lds_st(L, 1, l0.c1);
    lds_st(L, 4, l1.c0);
    lds_st(L, 5, l1.c1);
    lds_st(L, 6, l4.c0);
    lds_st(L, 7, l4.c1);
  }
}

// The loop as a schedule of phases: run(f) executes phase f for every lane of the workgroup (on the device: the
// calling lane, then a barrier; in the host model, tests/native/emu.cpp: lanes 0 .. GTW_MILLER_LANES - 1 in turn --
// within a phase no lane reads what another writes).
template <class Run>
BLS_INL void gtw_miller_schedule(Run&& run, uint32_t* F, const uint32_t* QA, const fp& xP, const fp& yP, uint32_t* TB,
                                 uint32_t* L0, uint32_t* L1, uint32_t* S, uint32_t* S2) {
  constexpr uint32_t TW = 64;  // lanes < TW: the T-chain wave; lane TW + i: f-lane i
  run([&](uint32_t t) {
    if (t < 6) lds_st(TB, (int)t, t < 4 ? lds_ld(QA, (int)t) : (t == 4 ? FP_ONE : fp_zero()));
    if (t < 12) lds_st(F, (int)t, t == 0 ? FP_ONE : fp_zero());
  });
  // the line of step 0 (a doubling)
  run([&](uint32_t t) {
    if (t < TW) gtw_dbl_p1(TB, S2, t);
  });
  run([&](uint32_t t) {
    if (t < TW) gtw_dbl_p2(TB, L0, S2, t);
  });
  run([&](uint32_t t) {
    if (t < TW) gtw_dbl_p3(TB, S2, xP, yP, t);
  });
  run([&](uint32_t t) {
    if (t < TW) gtw_dbl_p4(TB, L0, S2, t);
  });
  int bit = 61;
  bool add_next = (BLS_Z_ABS >> 62) & 1ull, cur_add = false;
#pragma unroll 1
  for (int s = 0; s < 68; s++) {
    uint32_t* cur = (s & 1) ? L1 : L0;
    uint32_t* nxt = (s & 1) ? L0 : L1;
    const bool more = s + 1 < 68, next_add = add_next;
    if (more) {
      if (next_add) {
        add_next = false;
      } else {
        add_next = (BLS_Z_ABS >> bit) & 1ull;
        bit--;
      }
    }
    const bool sq = !cur_add && s != 0;
    const bool dbl = more && !next_add;
    run([&](uint32_t t) {
      if (t >= TW) {
        if (sq) gtw_mul_prod<false>(F, F, S, t - TW);
      } else if (more) {
        if (next_add)
          gtw_add_step_lane(TB, QA, nxt, xP, yP, t);
        else
          gtw_dbl_p1(TB, S2, t);
      }
    });
    run([&](uint32_t t) {
      if (t >= TW) {
        if (sq) gtw_mul_rec<false>(F, S, t - TW);
      } else if (dbl) {
        gtw_dbl_p2(TB, nxt, S2, t);
      }
    });
    run([&](uint32_t t) {
      if (t >= TW)
        gtw_mul_prod<true>(F, cur, S, t - TW);
      else if (dbl)
        gtw_dbl_p3(TB, S2, xP, yP, t);
    });
    run([&](uint32_t t) {
      if (t >= TW)
        gtw_mul_rec<true>(F, S, t - TW);
      else if (dbl)
        gtw_dbl_p4(TB, nxt, S2, t);
    });
    cur_add = next_add;
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
  uint32_t S2[14 * BLS_NL];     // the Miller loop's T-chain products
  uint32_t TB[(6 + 14) * BLS_NL];  // T + doubling temporaries
  uint32_t QA[4 * BLS_NL];      // Q affine
  uint32_t flag;
};

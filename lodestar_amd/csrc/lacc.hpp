// Lazily reduced signed sums of Fp values for the cooperative GT engine (gt_wave.hpp): limb sums without carries,
// one carry pass and one quotient-estimate reduction at the end.  Host-compilable (tests/native/emu.cpp checks
// lacc_fin at the edges of its contract).
#pragma once
#include "fp.hpp"

// ---------------------------------------------------------------------------------------------------
// Lazily reduced signed sums of Fp values (each <= 2p, normalized limbs): limb sums without carries,
// one carry pass and one quotient-estimate reduction at the end.  At most 15 terms per side.
// ---------------------------------------------------------------------------------------------------
struct lacc {
  uint32_t pos[BLS_NL], neg[BLS_NL];
};
BLS_INL void lacc_init(lacc& a) {
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) a.pos[i] = a.neg[i] = 0;
}
BLS_INL void lacc_add(lacc& a, const fp& x) {
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) a.pos[i] += x.l[i];
}
BLS_INL void lacc_sub(lacc& a, const fp& x) {
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) a.neg[i] += x.l[i];
}
// 32 p in 28-bit limbs
BLS_INL uint32_t fp_p32_limb(int i) {
  uint32_t lo = (FP_P.l[i] << 5) & BLS_MASK;
  if (i == BLS_NL - 1) lo = FP_P.l[i] << 5;
  return lo | (i ? (FP_P.l[i - 1] >> (BLS_LB - 5)) : 0u);
}
// pos - neg (mod p), result <= 2p normalized
BLS_INL fp lacc_fin(const lacc& a) {
  uint32_t v[BLS_NL];
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) {
    int64_t d = (int64_t)a.pos[i] + (int64_t)fp_p32_limb(i) - (int64_t)a.neg[i] + c;
    if (i < BLS_NL - 1) {
      v[i] = (uint32_t)d & BLS_MASK;
      c = d >> BLS_LB;
    } else {
      v[i] = (uint32_t)d;  // value < 48 p < 2^387: top limb < 2^23
    }
  }
  // q = floor(vhi R / 2^57) with vhi = v's top 51 bits (limbs 13, 12) and R = floor(2^57 / (p's top 56 bits + 1)) =
  // 5040: never above floor(v / p) and at most 2 below (R's relative error is 2^-12.3 on quotients < 64), so
  // v - q p is in [0, 3p) and one conditional subtraction of p leaves [0, 2p).  (An integer multiply-shift: the
  // double-precision quotient this replaces cost ~0.4 us per call on one lane, tools/microbench/lat_probe.hip.)
  const uint64_t vhi = ((uint64_t)v[BLS_NL - 1] << BLS_LB) | v[BLS_NL - 2];
  const uint32_t q = (uint32_t)((vhi * 5040ull) >> 57);
  fp r;
  c = 0;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) {
    int64_t d = (int64_t)v[i] - (int64_t)((uint64_t)q * FP_P.l[i]) + c;
    if (i < BLS_NL - 1) {
      r.l[i] = (uint32_t)d & BLS_MASK;
      c = d >> BLS_LB;
    } else {
      r.l[i] = (uint32_t)d;
    }
  }
  return fp_csub_p(r);
}


// ---------------------------------------------------------------------------------------------------
// LDS access (Fp index q of a buffer: words q*14 .. q*14+13)
// ---------------------------------------------------------------------------------------------------
BLS_INL fp lds_ld(const uint32_t* b, int q) {
  fp r;
#pragma unroll
  for (int l = 0; l < BLS_NL; l++) r.l[l] = b[q * BLS_NL + l];
  return r;
}
BLS_INL void lds_st(uint32_t* b, int q, const fp& v) {
#pragma unroll
  for (int l = 0; l < BLS_NL; l++) b[q * BLS_NL + l] = v.l[l];
}

// a += coef * b[slot] (coef in -9 .. 9, as repeated terms)
BLS_INL void lacc_term(lacc& a, const uint32_t* b, int slot, int coef) {
  const fp v = lds_ld(b, slot);
  for (int k = 0; k < (coef < 0 ? -coef : coef); k++) {
    if (coef > 0)
      lacc_add(a, v);
    else
      lacc_sub(a, v);
  }
}
// a += coef * (component c of a Karatsuba Fp2 product whose three products P0, P1, P2 sit at slots k .. k + 2):
// c = 0: P0 - P1, c = 1: P2 - P0 - P1
BLS_INL void lacc_kara(lacc& a, const uint32_t* b, int k, int c, int coef) {
  if (c == 0) {
    lacc_term(a, b, k, coef);
    lacc_term(a, b, k + 1, -coef);
  } else {
    lacc_term(a, b, k + 2, coef);
    lacc_term(a, b, k, -coef);
    lacc_term(a, b, k + 1, -coef);
  }
}

// (x0 + x1 u)^2 = (x0 + x1)(x0 - x1) + (2 x0) x1 u : operands of component `comp`'s single product.  x0, x1:
// normalized limbs, values <= 4p; the operands are lazy (limbs < 2^30, values < 12p: fp_mul's contract)
BLS_INL void sqr_operands(const fp& x0, const fp& x1, int comp, fp& X, fp& Y) {
  X = comp ? fp_add_nr(x0, x0) : fp_add_nr(x0, x1);
  Y = comp ? x1 : fp_sub_k8(x0, x1);
}
// Karatsuba component c of (a0 + a1 u)(b0 + b1 u): c0 = a0 b0, c1 = a1 b1, c2 = (a0 + a1)(b0 + b1)
BLS_INL void kara_operands(const fp& a0, const fp& a1, const fp& b0, const fp& b1, int c, fp& X, fp& Y) {
  X = c == 0 ? a0 : (c == 1 ? a1 : fp_add_nr(a0, a1));
  Y = c == 0 ? b0 : (c == 1 ? b1 : fp_add_nr(b0, b1));
}


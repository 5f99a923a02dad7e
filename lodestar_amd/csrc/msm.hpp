// Bucket (Pippenger) multi-scalar multiplication for the signature side of the random linear combination:
//   S = sum_i r_i sig_i   over the included sets of one batch group (or of one job in the fallback)
// which blst computes inside verifyMultipleAggregateSignatures (reference maybeBatch.ts:17-38 ->
// @chainsafe/blst mul_n_aggregate).  Shared by the kernels (k_msm.hip) and the host build
// of the device arithmetic (tests/native/emu.cpp), which checks it against the oracle's sum of r_i sig_i.
//
// The batch scalar of a set is r = a + b lambda for its 64-bit word w (k_common.hpp jac_mul_scalar_word): a = sum_k
// d_k 16^k over the low 8 nibbles, b over the high 8, signed odd digits d_k = 2 nib_k(w) - 15 in {+-1, ..., +-15};
// w = 0 encodes r = 1 (CoreVerify of a single non-batchable set): a = 1 (low word 2^31: digits 1, -15, ..., -15) and
// no b part.  So window k of the MSM (k < 8: a, k >= 8: b) puts +-sig_i into bucket e = (|d_k| - 1) / 2 (8 buckets,
// no zero digit), and
//   S = S_a + lambda S_b,  S_a = sum_{k<8} 16^k W_k,  S_b = sum_{k<8} 16^k W_{8+k},  W_k = sum_e (2e + 1) B_{k,e}
// with lambda = -psi^2 on G2 (curve.hpp endo_lambda).  Per set this is 16 mixed additions (vs 28 doublings + 24
// additions of a per-set scalar multiplication); per range 16 bucket combinations (W_k) and two independent
// 8-window Horner passes (28 doublings + 7 additions each, on two lanes).
#pragma once
#include "curve.hpp"

#define MSM_WINDOWS 16
#define MSM_BUCKETS 8

#define MSM_NO_BUCKET 8u

// bucket of window k for scalar word w (MSM_NO_BUCKET: no term); neg = the digit is negative
BLS_HD uint32_t msm_bucket(uint64_t w, int k, bool& neg) {
  neg = false;
  if (w == 0) {
    if (k >= MSM_WINDOWS / 2) return MSM_NO_BUCKET;
    w = 1ull << 31;
  }
  const uint32_t nib = (uint32_t)(w >> (4 * k)) & 15u;
  neg = nib < 8;
  return neg ? 7u - nib : nib - 8u;
}

// W = sum_e (2e + 1) B_e on 8 lanes (k_msm_window): lane e forms (2e + 1) B_e with one chain for every lane (bits of e from the
// top, the addend T or infinity, so the wave does not diverge: 3 doublings + 3 additions), then a 3-level tree sums
// the 8 terms -- 6 additions deep instead of the 18 of running sums.
template <class F>
BLS_INL jac<F> msm_odd_multiple(const jac<F>& T, uint32_t e) {
  const jac<F> inf = jac_infinity<F>();
  jac<F> R = (e & 4u) ? T : inf;
  R = jac_add(jac_dbl(R), (e & 2u) ? T : inf);
  R = jac_add(jac_dbl(R), (e & 1u) ? T : inf);
  return jac_add(jac_dbl(R), T);
}
// host model of the 8-lane schedule (tests/native/emu.cpp): the same terms, the same tree
template <class LoadBucket>
BLS_INL g2j msm_window_sum_tree(LoadBucket bucket) {
  g2j v[MSM_BUCKETS];
  for (int e = 0; e < MSM_BUCKETS; e++) v[e] = msm_odd_multiple(bucket(e), (uint32_t)e);
  for (int h = 1; h < MSM_BUCKETS; h <<= 1)
    for (int e = 0; e < MSM_BUCKETS; e += 2 * h) v[e] = jac_add(v[e], v[e + h]);
  return v[0];
}

// half `part` of S: part 0 = S_a = sum_{k<8} 16^k W_k, part 1 = lambda S_b (Horner, most significant window first)
template <class LoadWindow>
BLS_INL g2j msm_horner_half(LoadWindow window, int part) {
  const int base = part * (MSM_WINDOWS / 2);
  g2j S = window(base + MSM_WINDOWS / 2 - 1);
#pragma unroll 1
  for (int k = MSM_WINDOWS / 2 - 2; k >= 0; k--) {
    S = jac_dbl(jac_dbl(jac_dbl(jac_dbl(S))));
    S = jac_add(S, window(base + k));
  }
  return part ? endo_lambda(S) : S;
}
// S = S_a + lambda S_b (one lane; the kernel runs the halves on two lanes)
template <class LoadWindow>
BLS_INL g2j msm_horner(LoadWindow window) {
  return jac_add(msm_horner_half(window, 0), msm_horner_half(window, 1));
}

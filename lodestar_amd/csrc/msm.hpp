// Bucket (Pippenger) multi-scalar multiplication for the signature side of the random linear combination:
//   S = sum_i r_i sig_i   over the included sets of one batch group (or of one job in the fallback)
// which blst computes inside verifyMultipleAggregateSignatures (reference maybeBatch.ts:17-38 ->
// @chainsafe/blst mul_n_aggregate).  Shared by the kernels (k_msm.hip) and the host build
// of the device arithmetic (tests/native/emu.cpp), which checks it against the oracle's sum of r_i sig_i.
//
// The batch scalar of a set is its 64-bit word w (runtime.cpp, k_common.hpp jac_mul_scalar_word): r = sum_k
// d_k 16^k over 16 signed odd digits d_k = 2 nib_k(w) - 15 in {+-1, +-3, ..., +-15}; w = 0 encodes r = 1
// (CoreVerify of a single non-batchable set), which is the word 2^63 (digits 1, -15, ..., -15).  So window k
// of the MSM puts +-sig_i into bucket e = (|d_k| - 1) / 2 (8 buckets, no zero digit), and
//   S = sum_k 16^k W_k,   W_k = sum_e (2e + 1) B_{k,e}.
// Per set this is 16 mixed additions (vs 61 doublings + 22 additions of a per-set scalar multiplication);
// per range 16 bucket combinations (W_k) and one Horner pass (60 doublings + 15 additions).
#pragma once
#include "curve.hpp"

#define MSM_WINDOWS 16
#define MSM_BUCKETS 8

// bucket of window k for scalar word w; neg = the digit is negative
BLS_HD uint32_t msm_bucket(uint64_t w, int k, bool& neg) {
  if (w == 0) w = 1ull << 63;
  const uint32_t nib = (uint32_t)(w >> (4 * k)) & 15u;
  neg = nib < 8;
  return neg ? 7u - nib : nib - 8u;
}

// W = sum_e (2e + 1) B_e by running sums:  acc_e = sum_{e' >= e} B_e',  tot = sum_e acc_e = sum_e (e + 1) B_e,
// W = 2 tot - acc_0.  `bucket(e)` yields B_e (Jacobian, possibly infinity).
template <class LoadBucket>
BLS_INL g2j msm_window_sum(LoadBucket bucket) {
  g2j acc = jac_infinity<fp2>(), tot = jac_infinity<fp2>();
#pragma unroll 1
  for (int e = MSM_BUCKETS - 1; e >= 0; e--) {
    acc = jac_add(acc, bucket(e));
    tot = jac_add(tot, acc);
  }
  return jac_add(jac_dbl(tot), jac_neg(acc));
}

// S = sum_k 16^k W_k (Horner, most significant window first)
template <class LoadWindow>
BLS_INL g2j msm_horner(LoadWindow window) {
  g2j S = window(MSM_WINDOWS - 1);
#pragma unroll 1
  for (int k = MSM_WINDOWS - 2; k >= 0; k--) {
    S = jac_dbl(jac_dbl(jac_dbl(jac_dbl(S))));
    S = jac_add(S, window(k));
  }
  return S;
}

// A9 signature side of the random linear combination, S = sum_i r_i sig_i per range (a batch group, or one
// job of the fallback), as a bucket multi-scalar multiplication (msm.hpp).  Three launches:
//   k_msm_bucket   one 128-lane workgroup per slice (<= MSM_SLICE sets of one range).  Lane t owns bucket
//                  (window k = t / 8, bucket e = t % 8).  Two counting passes over the slice's scalar words (in
//                  LDS) give every lane a compact list of its signed set indices (LDS, no atomics, so the order
//                  is deterministic); the lane then sums +-sig_i with mixed additions -> B[slice][t].  Lists keep
//                  the wave's lanes busy on useful additions: ~len/8 per lane instead of len masked ones.
//   k_msm_window   one lane per (range, window): W = sum_e (2e + 1) sum_{slices of the range} B_e
//   k_msm_horner   two lanes per range: S_a and lambda S_b (8-window Horner passes, msm.hpp), then S = their sum,
//                  written in the layout k_group_check reads
// Sets outside the batch equation (include == 0) and infinity signatures contribute nothing, as in the
// per-set scaling this replaces.
#include "k_common.hpp"
#include "msm.hpp"

#define MSM_LANES (MSM_WINDOWS * MSM_BUCKETS)

__global__ __launch_bounds__(MSM_LANES) __attribute__((amdgpu_waves_per_eu(BLSGPU_WPE_MSM, BLSGPU_WPE_MSM))) void k_msm_bucket(
    PipelineBuffers b, const uint32_t* slices, uint32_t n_slices, uint32_t* B) {
  __shared__ uint64_t sw[MSM_SLICE];
  __shared__ uint8_t act[MSM_SLICE];
  __shared__ uint16_t list[MSM_WINDOWS][MSM_SLICE];
  __shared__ uint16_t cnt[MSM_LANES];
  const uint32_t s = blockIdx.x, t = threadIdx.x;
  if (s >= n_slices) return;
  const uint32_t first = slices[2 * s], len = slices[2 * s + 1] - first;  // len <= MSM_SLICE (host)
  for (uint32_t j = t; j < len; j += MSM_LANES) {
    const uint32_t i = first + j;
    act[j] = b.include[i] && !(b.flags[i] & SF_SIG_INF);
    sw[j] = b.scalars[i];
  }
  __syncthreads();
  const int k = (int)(t / MSM_BUCKETS);
  const uint32_t e = t % MSM_BUCKETS;
  uint32_t c = 0;
  for (uint32_t j = 0; j < len; j++) {
    bool neg;
    c += (act[j] && msm_bucket(sw[j], k, neg) == e) ? 1u : 0u;
  }
  cnt[t] = (uint16_t)c;
  __syncthreads();
  uint32_t off = 0;
  for (uint32_t q = (uint32_t)k * MSM_BUCKETS; q < t; q++) off += cnt[q];
  for (uint32_t j = 0, p = off; j < len; j++) {
    bool neg;
    if (act[j] && msm_bucket(sw[j], k, neg) == e) list[k][p++] = (uint16_t)(j | (neg ? 0x8000u : 0u));
  }
  // each lane reads back only the entries it wrote: no barrier
  g2j acc = jac_infinity<fp2>();
#pragma unroll 1
  for (uint32_t q = 0; q < c; q++) {
    const uint32_t v = list[k][off + q];
    g2a P = ld_g2a(b.sig_aff, b.n, first + (v & 0x7fffu));
    if (v & 0x8000u) P.y = fp2_neg(P.y);
    acc = jac_add_aff(acc, P);
  }
  st_g2j(B, n_slices * MSM_LANES, s * MSM_LANES + t, acc);
}

// range r covers slices [range_slices[r], range_slices[r + 1])
STAGE_KERNEL void k_msm_window(const uint32_t* range_slices, uint32_t n_ranges, const uint32_t* B, uint32_t n_slices,
                               uint32_t* W) {
  const uint32_t q = blockIdx.x * WAVE + threadIdx.x;
  if (q >= n_ranges * MSM_WINDOWS) return;
  const uint32_t r = q / MSM_WINDOWS, k = q % MSM_WINDOWS;
  const uint32_t s0 = range_slices[r], s1 = range_slices[r + 1];
  const uint32_t nb = n_slices * MSM_LANES;
  const g2j Wk = msm_window_sum([&](int e) {
    g2j sum = jac_infinity<fp2>();
    for (uint32_t s = s0; s < s1; s++) sum = jac_add(sum, ld_g2j(B, nb, s * MSM_LANES + k * MSM_BUCKETS + e));
    return sum;
  });
  st_g2j(W, n_ranges * MSM_WINDOWS, q, Wk);
}

// lane pair (r, part) of one wave: part 1 leaves lambda S_b in its range's (already consumed) window-8 slot of W,
// part 0 adds it after the barrier.  W is written and read within the workgroup, so no lane returns early.
STAGE_KERNEL void k_msm_horner(uint32_t* W, uint32_t n_ranges, uint32_t* S) {
  const uint32_t q = blockIdx.x * WAVE + threadIdx.x;
  const uint32_t r = q >> 1, part = q & 1;
  const bool on = r < n_ranges;
  const uint32_t nw = n_ranges * MSM_WINDOWS;
  g2j H;
  if (on) {
    H = msm_horner_half([&](int k) { return ld_g2j(W, nw, r * MSM_WINDOWS + k); }, (int)part);
    if (part) st_g2j(W, nw, r * MSM_WINDOWS + MSM_WINDOWS / 2, H);
  }
  __syncthreads();
  if (on && !part) st_g2j(S, n_ranges, r, jac_add(H, ld_g2j(W, nw, r * MSM_WINDOWS + MSM_WINDOWS / 2)));
}

static inline dim3 grid_for(uint32_t n) { return dim3((n + WAVE - 1) / WAVE); }

void launch_sig_msm(const PipelineBuffers& b, const uint32_t* slices, uint32_t n_slices, const uint32_t* range_slices,
                    uint32_t n_ranges, uint32_t* B, uint32_t* W, uint32_t* S, hipStream_t st) {
  if (!n_ranges) return;
  if (n_slices) hipLaunchKernelGGL(k_msm_bucket, dim3(n_slices), dim3(MSM_LANES), 0, st, b, slices, n_slices, B);
  hipLaunchKernelGGL(k_msm_window, grid_for(n_ranges * MSM_WINDOWS), dim3(WAVE), 0, st, range_slices, n_ranges, B,
                     n_slices, W);
  hipLaunchKernelGGL(k_msm_horner, grid_for(2 * n_ranges), dim3(WAVE), 0, st, W, n_ranges, S);
}

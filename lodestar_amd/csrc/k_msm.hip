// A9 signature side of the random linear combination, S = sum_i r_i sig_i per range (a batch group, or one
// job of the fallback), as a bucket multi-scalar multiplication (msm.hpp).  Three launches:
//   k_msm_bucket   one 128-lane workgroup per slice (<= MSM_SLICE sets of one range).  Lane t owns bucket
//                  (window k = t / 8, bucket e = t % 8).  Two counting passes over the slice's scalar words (in
//                  LDS) give every lane a compact list of its signed set indices (LDS, no atomics, so the order
//                  is deterministic); the lane then sums +-sig_i with mixed additions -> B[slice][t].  Lists keep
//                  the wave's lanes busy on useful additions: ~len/8 per lane instead of len masked ones.
//   k_msm_window   eight lanes per (range, window): W = sum_e (2e + 1) sum_{slices of the range} B_e
//   k_msm_horner   two 16-lane groups per range: S_a and lambda S_b (8-window Horner passes, cooperative
//                  doublings), then S = their sum, written in the layout k_group_check reads
// Sets outside the batch equation (include == 0) and infinity signatures contribute nothing, as in the
// per-set scaling this replaces.
#include "k_common.hpp"
#include "msm.hpp"
#include "g2_coop.hpp"

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

// The bucket pass on lane pairs (fp2x.hpp): a 256-lane workgroup per slice, lane pair t / 2 owning bucket (window,
// e) and lane t holding coefficient t % 2 of its running sum -- half a point per lane, two waves per SIMD.  Both lanes
// of a pair build the same list (each reads back only what it wrote).
#ifndef BLSGPU_MSM_PAIRS
#define BLSGPU_MSM_PAIRS 1
#endif
// The window sums and the slice tree on lane pairs too: C2 within noise (3.72M vs 3.72M, three rounds of 100 steps),
// the isolated 16k call's MSM slower (3.7-4.2 vs 1.7-3.1 ms): off
#ifndef BLSGPU_MSM_WPAIRS
#define BLSGPU_MSM_WPAIRS 0
#endif
__global__ __launch_bounds__(2 * MSM_LANES) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_msm_bucket2(
    PipelineBuffers b, const uint32_t* slices, uint32_t n_slices, uint32_t* B) {
  __shared__ uint64_t sw[MSM_SLICE];
  __shared__ uint8_t act[MSM_SLICE];
  __shared__ uint16_t list[2][MSM_WINDOWS][MSM_SLICE];
  __shared__ uint16_t cnt[MSM_LANES];
  const uint32_t s = blockIdx.x, t = threadIdx.x, tb = t >> 1, kc = t & 1;
  if (s >= n_slices) return;
  const uint32_t first = slices[2 * s], len = slices[2 * s + 1] - first;  // len <= MSM_SLICE (host)
  for (uint32_t j = t; j < len; j += 2 * MSM_LANES) {
    const uint32_t i = first + j;
    act[j] = b.include[i] && !(b.flags[i] & SF_SIG_INF);
    sw[j] = b.scalars[i];
  }
  __syncthreads();
  const int k = (int)(tb / MSM_BUCKETS);
  const uint32_t e = tb % MSM_BUCKETS;
  uint32_t c = 0;
  for (uint32_t j = 0; j < len; j++) {
    bool neg;
    c += (act[j] && msm_bucket(sw[j], k, neg) == e) ? 1u : 0u;
  }
  if (kc == 0) cnt[tb] = (uint16_t)c;
  __syncthreads();
  uint32_t off = 0;
  for (uint32_t q = (uint32_t)k * MSM_BUCKETS; q < tb; q++) off += cnt[q];
  for (uint32_t j = 0, p = off; j < len; j++) {
    bool neg;
    if (act[j] && msm_bucket(sw[j], k, neg) == e) list[kc][k][p++] = (uint16_t)(j | (neg ? 0x8000u : 0u));
  }
  g2jx acc = jac_infinity<fp2x>();
#pragma unroll 1
  for (uint32_t q = 0; q < c; q++) {
    const uint32_t v = list[kc][k][off + q], i = first + (v & 0x7fffu);
    aff<fp2x> P;
    P.x.v = ld_fp(b.sig_aff, b.n, i, (int)(kc * W_FP));
    P.y.v = ld_fp(b.sig_aff, b.n, i, (int)((2 + kc) * W_FP));
    if (v & 0x8000u) P.y = F_neg(P.y);
    acc = jac_add_aff(acc, P);
  }
  st_g2jx(B, n_slices * MSM_LANES, s * MSM_LANES + tb, kc, acc);
}

// One lane per (range, window k, bucket e) -- the 8 lanes of a window are neighbours in one wave.  Range r covers
// slices [range_slices[r], range_slices[r + 1]); the lane sums its bucket over them (4 slices of a 16k call: 3
// additions), forms (2e + 1) B_e and the window's lanes sum their terms through LDS in a 3-level tree
// (msm_odd_multiple / msm_window_sum_tree): W_k in 3 + 6 additions + 3 doublings of depth instead of 3 x 8 + 18.
// One level of a pairwise tree over a range's slices (latency-bound runs with many short slices): lane per (range,
// pair j, bucket) adds slice s0 + (2j + 1) stride into slice s0 + 2j stride in place, so after ceil(log2(slices))
// levels the first slice of every range holds the range's bucket sums -- the window lanes' serial sum over 32 slices
// becomes 5 additions deep.
STAGE_KERNEL void k_msm_slice_pairs(const uint32_t* range_slices, uint32_t n_ranges, uint32_t* B, uint32_t n_slices,
                                    uint32_t stride, uint32_t max_pairs) {
  const uint32_t q = blockIdx.x * WAVE + threadIdx.x;
  const uint32_t tb = q % MSM_LANES, rest = q / MSM_LANES, j = rest % max_pairs, r = rest / max_pairs;
  if (r >= n_ranges) return;
  const uint32_t s0 = range_slices[r], s1 = range_slices[r + 1], a = s0 + 2 * j * stride, c = a + stride;
  if (c >= s1) return;
  const uint32_t nb = n_slices * MSM_LANES;
  st_g2j(B, nb, a * MSM_LANES + tb, jac_add(ld_g2j(B, nb, a * MSM_LANES + tb), ld_g2j(B, nb, c * MSM_LANES + tb)));
}

// the same level on lane pairs (fp2x.hpp)
STAGE_KERNEL_W(2) void k_msm_slice_pairs2(const uint32_t* range_slices, uint32_t n_ranges, uint32_t* B,
                                          uint32_t n_slices, uint32_t stride, uint32_t max_pairs) {
  const uint32_t q2 = blockIdx.x * WAVE + threadIdx.x, q = q2 >> 1, kc = q2 & 1;
  const uint32_t tb = q % MSM_LANES, rest = q / MSM_LANES, j = rest % max_pairs, r = rest / max_pairs;
  if (r >= n_ranges) return;
  const uint32_t s0 = range_slices[r], s1 = range_slices[r + 1], a = s0 + 2 * j * stride, c = a + stride;
  if (c >= s1) return;
  const uint32_t nb = n_slices * MSM_LANES;
  st_g2jx(B, nb, a * MSM_LANES + tb, kc,
          jac_add(ld_g2jx(B, nb, a * MSM_LANES + tb, kc), ld_g2jx(B, nb, c * MSM_LANES + tb, kc)));
}

STAGE_KERNEL void k_msm_window(const uint32_t* range_slices, uint32_t n_ranges, const uint32_t* B, uint32_t n_slices,
                               uint32_t* W, bool presummed) {
  __shared__ uint32_t xch[W_G2J * WAVE];
  const uint32_t t = threadIdx.x, q = blockIdx.x * WAVE + t;
  const bool on = q < n_ranges * MSM_LANES;
  const uint32_t r = q / MSM_LANES, tb = q % MSM_LANES, e = tb % MSM_BUCKETS;
  g2j T = jac_infinity<fp2>();
  if (on) {
    const uint32_t s0 = range_slices[r], s1 = presummed ? std::min(range_slices[r + 1], s0 + 1) : range_slices[r + 1],
                   nb = n_slices * MSM_LANES;
    if (s0 < s1) T = ld_g2j(B, nb, s0 * MSM_LANES + tb);
#pragma unroll 1
    for (uint32_t s = s0 + 1; s < s1; s++) T = jac_add(T, ld_g2j(B, nb, s * MSM_LANES + tb));
    T = msm_odd_multiple(T, e);
  }
  static_assert(WAVE % MSM_BUCKETS == 0, "a window's lanes share a workgroup");
#pragma unroll 1
  for (uint32_t h = 1; h < MSM_BUCKETS; h <<= 1) {
    if ((e & (2 * h - 1)) == h) st_g2j(xch, WAVE, t, T);
    __syncthreads();
    if ((e & (2 * h - 1)) == 0) T = jac_add(T, ld_g2j(xch, WAVE, t + h));
    __syncthreads();
  }
  if (on && e == 0) st_g2j(W, n_ranges * MSM_WINDOWS, q / MSM_BUCKETS, T);
}

// The window sums on lane pairs (fp2x.hpp): lane pair q / 2 per (range, window, bucket), lane q holding coefficient
// q % 2; the window's 16 lanes sum their terms through LDS in the same 3-level tree.
STAGE_KERNEL_W(2) void k_msm_window2(const uint32_t* range_slices, uint32_t n_ranges, const uint32_t* B,
                                     uint32_t n_slices, uint32_t* W, bool presummed) {
  __shared__ uint32_t xch[3 * W_FP * WAVE];
  const uint32_t t = threadIdx.x, q = blockIdx.x * WAVE + t, qb = q >> 1, kc = q & 1;
  const bool on = qb < n_ranges * MSM_LANES;
  const uint32_t r = qb / MSM_LANES, tb = qb % MSM_LANES, e = tb % MSM_BUCKETS;
  g2jx T = jac_infinity<fp2x>();
  if (on) {
    const uint32_t s0 = range_slices[r], s1 = presummed ? std::min(range_slices[r + 1], s0 + 1) : range_slices[r + 1],
                   nb = n_slices * MSM_LANES;
    if (s0 < s1) T = ld_g2jx(B, nb, s0 * MSM_LANES + tb, kc);
#pragma unroll 1
    for (uint32_t s = s0 + 1; s < s1; s++) T = jac_add(T, ld_g2jx(B, nb, s * MSM_LANES + tb, kc));
    T = msm_odd_multiple(T, e);
  }
  static_assert(WAVE % (2 * MSM_BUCKETS) == 0, "a window's lane pairs share a workgroup");
#pragma unroll 1
  for (uint32_t h = 1; h < MSM_BUCKETS; h <<= 1) {
    if ((e & (2 * h - 1)) == h) {
      st_fp(xch, WAVE, t, 0, T.x.v);
      st_fp(xch, WAVE, t, W_FP, T.y.v);
      st_fp(xch, WAVE, t, 2 * W_FP, T.z.v);
    }
    __syncthreads();
    if ((e & (2 * h - 1)) == 0) {
      g2jx o;
      o.x.v = ld_fp(xch, WAVE, t + 2 * h, 0);
      o.y.v = ld_fp(xch, WAVE, t + 2 * h, W_FP);
      o.z.v = ld_fp(xch, WAVE, t + 2 * h, 2 * W_FP);
      T = jac_add(T, o);
    }
    __syncthreads();
  }
  if (on && e == 0) st_g2jx(W, n_ranges * MSM_WINDOWS, qb / MSM_BUCKETS, kc, T);
}

// Horner passes on cooperative 16-lane groups (g2_coop.hpp): a workgroup of 128 lanes runs 4 ranges, group 2j the
// S_a pass of range 4 blockIdx + j, group 2j + 1 its lambda S_b pass; the 28 doublings and 7 window additions of a
// pass are cooperative (lambda on the group's lane 0), then group 2j adds its neighbour's lambda S_b the same way.
#define MSM_H_LANES 128
#define MSM_H_RANGES (MSM_H_LANES / G2C_LANES / 2)
__global__ __launch_bounds__(MSM_H_LANES) void k_msm_horner(const uint32_t* W, uint32_t n_ranges, uint32_t* S) {
  __shared__ uint32_t lds[(MSM_H_LANES / G2C_LANES) * G2C_WORDS];
  const uint32_t t = threadIdx.x, grp = t / G2C_LANES, tg = t % G2C_LANES;
  const uint32_t r = blockIdx.x * MSM_H_RANGES + grp / 2, part = grp & 1;
  const bool on = r < n_ranges;
  const uint32_t nw = n_ranges * MSM_WINDOWS, base = r * MSM_WINDOWS + part * (MSM_WINDOWS / 2);
  uint32_t* g = lds + grp * G2C_WORDS;
  if (tg == 0) g2c_st_point(g, on ? ld_g2j(W, nw, base + MSM_WINDOWS / 2 - 1) : jac_infinity<fp2>());
  g2c_sync();
#pragma unroll 1
  for (int k = MSM_WINDOWS / 2 - 2; k >= 0; k--) {
#pragma unroll 1
    for (int d = 0; d < 4; d++) g2c_dbl(g, tg);
    if (tg == 0 && on) g2c_st_q(g, ld_g2j(W, nw, base + (uint32_t)k));
    g2c_sync();
    g2c_add(g, tg, on);
  }
  if (tg == 0 && on && part) g2c_st_point(g, endo_lambda(g2c_ld_point(g)));
  g2c_sync();
  if (tg == 0 && on && !part) g2c_st_q(g, g2c_ld_point(g + G2C_WORDS));
  g2c_sync();
  g2c_add(g, tg, on && !part);
  if (tg == 0 && on && !part) st_g2j(S, n_ranges, r, g2c_ld_point(g));
}

// The same two Horner passes on two LANES per range (lane 2r: S_a, lane 2r + 1: lambda S_b, then lane 2r adds its
// partner's result through a lane exchange) -- for merged runs, where the chip is full of one-wave-per-SIMD stage
// kernels: a 128-lane cooperative workgroup needs two free SIMDs of one CU at once and waited ~16 ms for them in the
// driver's trace (the signature branch was the run's critical path); single waves take any free SIMD.
STAGE_KERNEL void k_msm_horner_lane(const uint32_t* W, uint32_t n_ranges, uint32_t* S) {
  const uint32_t q = blockIdx.x * WAVE + threadIdx.x;
  const uint32_t r = q >> 1, part = q & 1;
  if (r >= n_ranges) return;  // both lanes of a pair leave together (WAVE is even)
  const uint32_t nw = n_ranges * MSM_WINDOWS;
  const g2j h = msm_horner_half([&](int k) { return ld_g2j(W, nw, r * MSM_WINDOWS + (uint32_t)k); }, (int)part);
  const g2j o = g2j_xlane(h);
  if (!part) st_g2j(S, n_ranges, r, jac_add(h, o));
}

static inline dim3 grid_for(uint32_t n) { return dim3((n + WAVE - 1) / WAVE); }

void launch_sig_msm(const PipelineBuffers& b, const uint32_t* slices, uint32_t n_slices, const uint32_t* range_slices,
                    uint32_t n_ranges, uint32_t* B, uint32_t* W, uint32_t* S, hipStream_t st, bool lane_tail,
                    uint32_t tree_slices) {
  if (!n_ranges) return;
  if (n_slices) {
    if (BLSGPU_MSM_PAIRS)
      hipLaunchKernelGGL(k_msm_bucket2, dim3(n_slices), dim3(2 * MSM_LANES), 0, st, b, slices, n_slices, B);
    else
      hipLaunchKernelGGL(k_msm_bucket, dim3(n_slices), dim3(MSM_LANES), 0, st, b, slices, n_slices, B);
  }
  const bool tree = n_slices && tree_slices > 2;
  if (tree)
    for (uint32_t stride = 1; stride < tree_slices; stride *= 2) {
      const uint32_t max_pairs = (tree_slices + 2 * stride - 1) / (2 * stride);
      if (BLSGPU_MSM_WPAIRS)
        hipLaunchKernelGGL(k_msm_slice_pairs2, grid_for(2 * n_ranges * max_pairs * MSM_LANES), dim3(WAVE), 0, st,
                           range_slices, n_ranges, B, n_slices, stride, max_pairs);
      else
        hipLaunchKernelGGL(k_msm_slice_pairs, grid_for(n_ranges * max_pairs * MSM_LANES), dim3(WAVE), 0, st,
                           range_slices, n_ranges, B, n_slices, stride, max_pairs);
    }
  if (BLSGPU_MSM_WPAIRS)
    hipLaunchKernelGGL(k_msm_window2, grid_for(2 * n_ranges * MSM_LANES), dim3(WAVE), 0, st, range_slices, n_ranges, B,
                       n_slices, W, tree);
  else
    hipLaunchKernelGGL(k_msm_window, grid_for(n_ranges * MSM_LANES), dim3(WAVE), 0, st, range_slices, n_ranges, B,
                       n_slices, W, tree);
  if (lane_tail)
    hipLaunchKernelGGL(k_msm_horner_lane, grid_for(2 * n_ranges), dim3(WAVE), 0, st, W, n_ranges, S);
  else
    hipLaunchKernelGGL(k_msm_horner, dim3((n_ranges + MSM_H_RANGES - 1) / MSM_H_RANGES), dim3(MSM_H_LANES), 0, st, W,
                       n_ranges, S);
}

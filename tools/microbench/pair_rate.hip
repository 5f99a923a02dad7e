// Chip throughput of the one-lane Fp2 forms (one wave per SIMD, the whole register file) against the lane-pair forms
// (fp2x.hpp / gtx.hpp, two waves per SIMD), on the shapes the stage kernels run:
//   dbl   G2 Jacobian doublings (curve.hpp jac_dbl), the [|z|] chains of the cofactor clearing / subgroup check
//   acc   Miller accumulation steps: f = fp12_sqr(f) * line (tower.hpp fp12_sqr + fp12_mul_by_014)
//   mul   independent Fp2 products (two chains per lane)
// Each variant runs WAVES_PER_SIMD x 1,024 SIMDs x ROUNDS waves; a "unit" is one doubling / one accumulation step /
// one Fp2 product of one item (a lane for one-lane forms, a lane pair for pair forms).  The pair results are checked
// against the one-lane results (same seeds), so the microbenchmark also pins gtx.hpp's formulas.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include tools/microbench/pair_rate.hip -o tools/microbench/pair_rate
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../lodestar_amd/csrc/gtx.hpp"
#include "../../lodestar_amd/csrc/tower.hpp"

constexpr int ITERS = 16;
constexpr int ROUNDS = 4;

__device__ __forceinline__ fp seed_fp(uint32_t t, uint32_t k) {
  fp a;
  for (int i = 0; i < BLS_NL; i++) a.l[i] = (t * (7919u + 2 * k) + i * (104729u + 31 * k) + 12345u * k) & BLS_MASK;
  a.l[BLS_NL - 1] &= 0xFFFu;  // value < p
  return a;
}
__device__ __forceinline__ fp2 seed_fp2(uint32_t t, uint32_t k) { return fp2_make(seed_fp(t, 2 * k), seed_fp(t, 2 * k + 1)); }

template <class F>
struct Out;

// one-lane forms: item = lane.  out[item * 12 + j][l] canonical words of the result's Fp components
template <int V>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1))) void k_one(uint32_t* out, uint32_t n_items) {
  const uint32_t item = blockIdx.x * 64 + threadIdx.x;
  if (item >= n_items) return;
  const uint32_t sd = item % 4096;
  if constexpr (V == 0) {
    g2j p;
    p.x = seed_fp2(sd, 0);
    p.y = seed_fp2(sd, 1);
    p.z = seed_fp2(sd, 2);
#pragma unroll 1
    for (int it = 0; it < ITERS; it++) p = jac_dbl(p);
    const fp* w = &p.x.c0;
    for (int j = 0; j < 6; j++) {
      const fp c = fp_canon(w[j]);
      for (int l = 0; l < BLS_NL; l++) out[((size_t)item * 12 + j) * BLS_NL + l] = c.l[l];
    }
  } else if constexpr (V == 1) {
    fp12 f;
    fp2* w = &f.c0.c0;
    for (int j = 0; j < 6; j++) w[j] = seed_fp2(sd, j);
    const fp2 l0 = seed_fp2(sd, 7), l1 = seed_fp2(sd, 8), l4 = seed_fp2(sd, 9);
#pragma unroll 1
    for (int it = 0; it < ITERS; it++) f = fp12_mul_by_014(fp12_sqr(f), l0, l1, l4);
    for (int j = 0; j < 6; j++) {
      const fp c0 = fp_canon(w[j].c0), c1 = fp_canon(w[j].c1);
      for (int l = 0; l < BLS_NL; l++) {
        out[((size_t)item * 12 + 2 * j) * BLS_NL + l] = c0.l[l];
        out[((size_t)item * 12 + 2 * j + 1) * BLS_NL + l] = c1.l[l];
      }
    }
  } else {
    fp2 a = seed_fp2(sd, 0), b = seed_fp2(sd, 1), c = seed_fp2(sd, 2);
#pragma unroll 1
    for (int it = 0; it < ITERS * 8; it++) {
      a = fp2_mul(a, c);
      b = fp2_mul(b, c);
    }
    const fp x = fp_canon(fp_add(a.c0, b.c1));
    for (int l = 0; l < BLS_NL; l++) out[((size_t)item * 12) * BLS_NL + l] = x.l[l];
  }
}

// pair forms: item = lane pair, lane k holds coefficient k
template <int V>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_pair(uint32_t* out, uint32_t n_items) {
  const uint32_t q = blockIdx.x * 64 + threadIdx.x, item = q >> 1, k = q & 1;
  if (item >= n_items) return;
  const uint32_t sd = item % 4096;
  auto co = [&](const fp2& v) { return fp2x{k ? v.c1 : v.c0}; };
  if constexpr (V == 0) {
    g2jx p;
    p.x = co(seed_fp2(sd, 0));
    p.y = co(seed_fp2(sd, 1));
    p.z = co(seed_fp2(sd, 2));
#pragma unroll 1
    for (int it = 0; it < ITERS; it++) p = jac_dbl(p);
    const fp2x* w = &p.x;
    for (int j = 0; j < 3; j++) {
      const fp c = fp_canon(w[j].v);
      for (int l = 0; l < BLS_NL; l++) out[((size_t)item * 12 + 2 * j + k) * BLS_NL + l] = c.l[l];
    }
  } else if constexpr (V == 1) {
    fp12x f;
    fp2x* w = &f.c0.c0;
    for (int j = 0; j < 6; j++) w[j] = co(seed_fp2(sd, j));
    const fp2x l0 = co(seed_fp2(sd, 7)), l1 = co(seed_fp2(sd, 8)), l4 = co(seed_fp2(sd, 9));
#pragma unroll 1
    for (int it = 0; it < ITERS; it++) f = fp12x_mul_by_014(fp12x_sqr(f), l0, l1, l4);
    for (int j = 0; j < 6; j++) {
      const fp c = fp_canon(w[j].v);
      for (int l = 0; l < BLS_NL; l++) out[((size_t)item * 12 + 2 * j + k) * BLS_NL + l] = c.l[l];
    }
  } else {
    fp2x a = co(seed_fp2(sd, 0)), b = co(seed_fp2(sd, 1)), c = co(seed_fp2(sd, 2));
#pragma unroll 1
    for (int it = 0; it < ITERS * 8; it++) {
      a = F_mul(a, c);
      b = F_mul(b, c);
    }
    // x = a.c0 + b.c1: lane 0 holds a.c0, lane 1 b.c1
    const fp mine = k ? b.v : a.v;
    const fp x = fp_canon(fp_add(mine, fp_swap(mine)));
    if (k == 0)
      for (int l = 0; l < BLS_NL; l++) out[((size_t)item * 12) * BLS_NL + l] = x.l[l];
  }
}

#define CHK(x)                                                              \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
      exit(1);                                                              \
    }                                                                       \
  } while (0)

template <class K>
static double run(K kern, int lanes_per_item, int wpe, uint32_t* d_out, uint32_t& n_items_out) {
  const uint32_t waves = 1024u * wpe * ROUNDS;
  const uint32_t n_items = waves * 64 / lanes_per_item;
  n_items_out = n_items;
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  hipLaunchKernelGGL(kern, dim3(waves), dim3(64), 0, 0, d_out, n_items);  // warm
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(a, 0));
  hipLaunchKernelGGL(kern, dim3(waves), dim3(64), 0, 0, d_out, n_items);
  CHK(hipEventRecord(b, 0));
  CHK(hipEventSynchronize(b));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, a, b));
  return ms;
}

int main() {
  const size_t words = (size_t)1024 * 2 * ROUNDS * 64 * 12 * BLS_NL;
  uint32_t *d1, *d2;
  CHK(hipMalloc(&d1, words * 4));
  CHK(hipMalloc(&d2, words * 4));
  uint32_t* h1 = (uint32_t*)malloc(words * 4);
  uint32_t* h2 = (uint32_t*)malloc(words * 4);
  const char* names[3] = {"dbl", "acc", "mul"};
  const int units_per_item[3] = {ITERS, ITERS, 2 * 8 * ITERS};
  printf("{\"tool\": \"tools/microbench/pair_rate.hip\", \"iters\": %d, \"rounds\": %d, \"results\": [\n", ITERS, ROUNDS);
  for (int v = 0; v < 3; v++) {
    uint32_t n1 = 0, n2 = 0;
    CHK(hipMemset(d1, 0, words * 4));
    CHK(hipMemset(d2, 0, words * 4));
    double ms1 = v == 0 ? run(k_one<0>, 1, 1, d1, n1) : v == 1 ? run(k_one<1>, 1, 1, d1, n1) : run(k_one<2>, 1, 1, d1, n1);
    double ms2 = v == 0 ? run(k_pair<0>, 2, 2, d2, n2) : v == 1 ? run(k_pair<1>, 2, 2, d2, n2) : run(k_pair<2>, 2, 2, d2, n2);
    CHK(hipMemcpy(h1, d1, words * 4, hipMemcpyDeviceToHost));
    CHK(hipMemcpy(h2, d2, words * 4, hipMemcpyDeviceToHost));
    // compare the items both ran (seeded by item % 4096): the first min(n1, n2) items
    const uint32_t n = n1 < n2 ? n1 : n2;
    const int comps = v == 2 ? 1 : (v == 0 ? 6 : 12);
    size_t bad = 0;
    for (uint32_t i = 0; i < n; i++)
      for (int j = 0; j < comps; j++)
        if (memcmp(h1 + ((size_t)i * 12 + j) * BLS_NL, h2 + ((size_t)i * 12 + j) * BLS_NL, BLS_NL * 4)) bad++;
    const double r1 = (double)n1 * units_per_item[v] / (ms1 * 1e-3), r2 = (double)n2 * units_per_item[v] / (ms2 * 1e-3);
    printf("  {\"shape\": \"%s\", \"one_lane_units_per_s\": %.4g, \"pair_units_per_s\": %.4g, \"pair_over_one\": %.3f, "
           "\"one_ms\": %.3f, \"pair_ms\": %.3f, \"mismatched_components\": %zu}%s\n",
           names[v], r1, r2, r2 / r1, ms1, ms2, bad, v < 2 ? "," : "");
  }
  printf("]}\n");
  return 0;
}

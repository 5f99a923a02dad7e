// A11 hash_to_G2 of every set's signing root, one lane per set.
#include "k_common.hpp"

STAGE_KERNEL void k_hash_to_g2(PipelineBuffers b, uint32_t n_sets) {
  uint32_t i = blockIdx.x * WAVE + threadIdx.x;
  if (i >= n_sets) return;
  uint8_t msg[32];
  const uint4* src = reinterpret_cast<const uint4*>(b.msgs + (size_t)i * 32);
  uint4 m0 = src[0], m1 = src[1];
  uint32_t w[8] = {m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w};
#pragma unroll
  for (int k = 0; k < 32; k++) msg[k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
  g2j h = hash_to_g2_jac(msg);
  g2a a;
  bool ok = jac_to_aff(h, a);
  if (!ok) {
    a.x = fp2_zero();
    a.y = fp2_zero();
  }
  st_g2a(b.h_aff, b.n, i, a);
  b.flags[b.n + i] = ok ? 0 : SF_H_INF;  // hash flags: flags[n, 2n)
}

static inline dim3 grid_for(uint32_t n) { return dim3((n + WAVE - 1) / WAVE); }

void launch_hash_to_g2(const PipelineBuffers& b, uint32_t n, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_hash_to_g2, grid_for(n), dim3(WAVE), 0, s, b, n);
}

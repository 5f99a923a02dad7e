// A11 hash_to_G2, one lane per DISTINCT signing root of the call (the runtime deduplicates messages: gossip
// attestations of one committee share AttestationData, reference chain/validation/attestation.ts:131-138).
#include "k_common.hpp"

STAGE_KERNEL void k_hash_to_g2(PipelineBuffers b) {
  uint32_t u = blockIdx.x * WAVE + threadIdx.x;
  if (u >= b.n_umsg) return;
  uint8_t msg[32];
  const uint4* src = reinterpret_cast<const uint4*>(b.umsgs + (size_t)u * 32);
  uint4 m0 = src[0], m1 = src[1];
  uint32_t w[8] = {m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w};
#pragma unroll
  for (int k = 0; k < 32; k++) msg[k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
  // Jacobian out; the affine conversion is batched over the messages (k_inv.hip k_h_affine)
  const g2j h = hash_to_g2_jac(msg);
  st_g2j(b.h_jac, b.nm, u, h);
  st_fp(b.h_norm, b.nm, u, 0, fp2_norm(h.z));
}

static inline dim3 grid_for(uint32_t n) { return dim3((n + WAVE - 1) / WAVE); }

void launch_hash_to_g2(const PipelineBuffers& b, hipStream_t s) {
  if (b.n_umsg) hipLaunchKernelGGL(k_hash_to_g2, grid_for(b.n_umsg), dim3(WAVE), 0, s, b);
}

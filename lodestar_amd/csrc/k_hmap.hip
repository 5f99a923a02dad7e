// A11 hash_to_G2, hash_to_field and the SSWU maps + isogeny (k_hash.hip describes the stage).  Their own translation
// unit: the callees (SHA-256, the (p-3)/4 exponentiations, the product calls) are then reached from two-wave kernels
// only, so the register budget of two waves per SIMD reaches them too (shared with k_hash_clear's one-lane form they
// were compiled for the one-wave budget and both kernels stayed at one wave).  The exponentiations dominate the maps
// and need few registers; the Fp2 state around them is saved once per call.
#include "k_common.hpp"

#define W_HPREP (7 * 2 * W_FP)

__device__ __forceinline__ void st_prep(uint32_t* p, uint32_t n, uint32_t u, const h2c_prep& h) {
  st_fp2(p, n, u, 0 * W_FP, h.u0);
  st_fp2(p, n, u, 2 * W_FP, h.u1);
  st_fp2(p, n, u, 4 * W_FP, h.Zu2_0);
  st_fp2(p, n, u, 6 * W_FP, h.Zu2_1);
  st_fp2(p, n, u, 8 * W_FP, h.tv0);
  st_fp2(p, n, u, 10 * W_FP, h.tv1);
  st_fp2(p, n, u, 12 * W_FP, h.d);
}
STAGE_KERNEL_W(BLSGPU_WPE_HPREP) void k_hash_prep(PipelineBuffers b) {
  uint32_t u = blockIdx.x * WAVE + threadIdx.x;
  if (u >= b.n_umsg) return;
  uint8_t msg[32];
  const uint4* src = reinterpret_cast<const uint4*>(b.umsgs + (size_t)u * 32);
  uint4 m0 = src[0], m1 = src[1];
  uint32_t w[8] = {m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w};
#pragma unroll
  for (int k = 0; k < 32; k++) msg[k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
  h2c_prep h;
  hash_to_g2_prep(msg, h);
  st_prep(b.h_prep, b.nm, u, h);
  st_fp(b.h_norm, b.nm, u, 0, fp2_norm(h.d));
}

__device__ __forceinline__ h2c_prep ld_prep(const uint32_t* p, uint32_t n, uint32_t u) {
  h2c_prep h;
  h.u0 = ld_fp2(p, n, u, 0 * W_FP);
  h.u1 = ld_fp2(p, n, u, 2 * W_FP);
  h.Zu2_0 = ld_fp2(p, n, u, 4 * W_FP);
  h.Zu2_1 = ld_fp2(p, n, u, 6 * W_FP);
  h.tv0 = ld_fp2(p, n, u, 8 * W_FP);
  h.tv1 = ld_fp2(p, n, u, 10 * W_FP);
  h.d = ld_fp2(p, n, u, 12 * W_FP);
  return h;
}

// inv: 1 / N(d) from the batch inversion; d^-1 = conj(d) / N(d).  Two lanes per message (lane pair (u, j)): each
// runs one SSWU map + isogeny -> h_q[j] (the two maps of a message are independent, so a small call's hash
// latency drops by one map).
STAGE_KERNEL_W(BLSGPU_WPE_HMAP) void k_hash_map(PipelineBuffers b, const uint32_t* inv) {
  const uint32_t q = blockIdx.x * WAVE + threadIdx.x;
  if (q >= 2 * b.n_umsg) return;
  const uint32_t u = q >> 1, j = q & 1;
  const h2c_prep h = ld_prep(b.h_prep, b.nm, u);
  const fp ni = ld_fp(inv, b.n_umsg, u, 0);
  const fp2 dinv = fp2_make(fp_mul(h.d.c0, ni), fp_neg(fp_mul(h.d.c1, ni)));
  st_g2j(b.h_q, 2 * b.nm, q, hash_to_g2_map_j(h, dinv, (int)j));
}

void launch_hash_prep(const PipelineBuffers& b, hipStream_t s) {
  if (b.n_umsg) hipLaunchKernelGGL(k_hash_prep, dim3((b.n_umsg + WAVE - 1) / WAVE), dim3(WAVE), 0, s, b);
}
void launch_hash_map(const PipelineBuffers& b, const uint32_t* inv, hipStream_t s) {
  if (b.n_umsg) hipLaunchKernelGGL(k_hash_map, dim3((2 * b.n_umsg + WAVE - 1) / WAVE), dim3(WAVE), 0, s, b, inv);
}

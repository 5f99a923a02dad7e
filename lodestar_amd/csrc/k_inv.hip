// Simultaneous (Montgomery-trick) inversion for the affine conversions of the pipeline.
//
// In SIMT a per-lane inversion costs the wave one full exponentiation (~460 Montgomery products) whatever
// the lanes do, so inverting per set is as expensive as it looks.  Here one lane inverts a slice of
// INV_K elements with ONE exponentiation and 3 products per element: prefix products forward, one
// inversion, then the inverses backward.  Lane l owns elements l, l + L, l + 2L, ... (L = lane count), so
// every SoA load and store stays coalesced.  A zero element is skipped in the chain and gets 0 back.
//
// Users (each replaces a per-lane jac_to_aff):
//   k_pk_affine  r_i pk_i: Jacobian (k_pk_finish) -> affine P of the Miller loop (pk_aff)
//   k_h_affine   H(m):     Jacobian (k_hash_to_g2) -> affine Q of the Miller lines (h_aff); the Fp2
//                          inversion goes through the norm, 1/z = conj(z) / N(z), so the batch is in Fp.
#include "k_common.hpp"

#define INV_K 16

// dst[i] = 1 / src[i] (0 -> 0) for i < n; src element i at src[(w0 + l) * src_stride + i], dst SoA stride n.
// dst also holds the prefix products between the two passes.
__global__ __launch_bounds__(WAVE) void k_batch_inv(const uint32_t* src, uint32_t src_stride, int w0, uint32_t* dst,
                                                    uint32_t n, uint32_t lanes) {
  const uint32_t l = blockIdx.x * WAVE + threadIdx.x;
  if (l >= lanes) return;
  fp acc = FP_ONE;
#pragma unroll 1
  for (uint32_t j = 0; j < INV_K; j++) {
    const uint32_t i = l + j * lanes;
    if (i >= n) break;
    const fp z = ld_fp(src, src_stride, i, w0);
    st_fp(dst, n, i, 0, acc);  // product of the slice's earlier nonzero elements
    if (!fp_is_zero(z)) acc = fp_mul(acc, z);
  }
  fp inv = fp_inv(acc);
#pragma unroll 1
  for (int j = INV_K - 1; j >= 0; j--) {
    const uint32_t i = l + (uint32_t)j * lanes;
    if (i >= n) continue;
    const fp z = ld_fp(src, src_stride, i, w0);
    const bool zero = fp_is_zero(z);
    const fp zi = fp_mul(inv, ld_fp(dst, n, i, 0));
    if (!zero) inv = fp_mul(inv, z);
    st_fp(dst, n, i, 0, zero ? fp_zero() : zi);
  }
}

// r_i pk_i (Jacobian, pk_jac) -> affine pk_aff with the batch inverses of the z coordinates (inv).  A point at
// infinity turns a clean set's pubkey status into PK_IS_INFINITY (as the per-lane jac_to_aff did).
__global__ __launch_bounds__(WAVE) void k_pk_affine(PipelineBuffers b, uint32_t n_sets, const uint32_t* inv,
                                                    int8_t* pk_status) {
  const uint32_t i = blockIdx.x * WAVE + threadIdx.x;
  if (i >= n_sets) return;
  g1a out;
  out.x = fp_zero();
  out.y = fp_zero();
  if (pk_status[i] == BLS_OK) {
    const g1j R = ld_g1j(b.pk_jac, b.n, i);
    if (jac_is_inf(R)) {
      pk_status[i] = BLS_PK_IS_INFINITY;
    } else {
      const fp zi = ld_fp(inv, n_sets, i, 0);
      const fp zi2 = fp_sqr(zi);
      out.x = fp_mul(R.x, zi2);
      out.y = fp_mul(R.y, fp_mul(zi2, zi));
    }
  }
  st_g1a(b.pk_aff, b.n, i, out);
}

// H(m) (Jacobian, h_jac) -> affine h_aff; inv holds 1 / N(z).  Infinity -> MF_H_INF (pairs to 1).
__global__ __launch_bounds__(WAVE) void k_h_affine(PipelineBuffers b, const uint32_t* inv) {
  const uint32_t u = blockIdx.x * WAVE + threadIdx.x;
  if (u >= b.n_umsg) return;
  const g2j h = ld_g2j(b.h_jac, b.nm, u);
  g2a a;
  a.x = fp2_zero();
  a.y = fp2_zero();
  const bool inf = jac_is_inf(h);
  if (!inf) {
    const fp ni = ld_fp(inv, b.n_umsg, u, 0);
    const fp2 zi = fp2_make(fp_mul(h.z.c0, ni), fp_neg(fp_mul(h.z.c1, ni)));  // conj(z) / N(z)
    const fp2 zi2 = fp2_sqr(zi);
    a.x = fp2_mul(h.x, zi2);
    a.y = fp2_mul(h.y, fp2_mul(zi2, zi));
  }
  st_g2a(b.h_aff, b.nm, u, a);
  b.mflags[u] = inf ? MF_H_INF : 0;
}

static inline dim3 grid_for(uint32_t n) { return dim3((n + WAVE - 1) / WAVE); }

void launch_batch_inv(const uint32_t* src, uint32_t src_stride, int w0, uint32_t* dst, uint32_t n, hipStream_t s) {
  if (!n) return;
  // up to 16k elements (one wave per SIMD at most; small and medium runs, latency first): one element per lane,
  // the inversion without the prefix chains (~0.1 ms instead of ~0.2 ms on each branch of a call that inverts)
  const uint32_t lanes = n <= 16384 ? n : (n + INV_K - 1) / INV_K;
  hipLaunchKernelGGL(k_batch_inv, grid_for(lanes), dim3(WAVE), 0, s, src, src_stride, w0, dst, n, lanes);
}
void launch_pk_affine(const PipelineBuffers& b, uint32_t n, hipStream_t s) {
  if (!n) return;
  uint32_t* inv = b.inv_buf_pk ? b.inv_buf_pk : b.inv_buf;
  launch_batch_inv(b.pk_jac, b.n, 2 * W_FP, inv, n, s);
  hipLaunchKernelGGL(k_pk_affine, grid_for(n), dim3(WAVE), 0, s, b, n, inv, b.status + b.n);
}
void launch_h_affine(const PipelineBuffers& b, hipStream_t s) {
  if (!b.n_umsg) return;
  launch_batch_inv(b.h_norm, b.nm, 0, b.inv_buf, b.n_umsg, s);
  hipLaunchKernelGGL(k_h_affine, grid_for(b.n_umsg), dim3(WAVE), 0, s, b, b.inv_buf);
}

// A12 per-set Miller loops f_i = MillerLoop(r_i pk_i, H(m_i)), one lane per set.
#include "k_common.hpp"

__global__ __launch_bounds__(WAVE) void k_miller_sets(PipelineBuffers b, uint32_t n_sets, const int8_t* pk_status) {
  uint32_t i = blockIdx.x * WAVE + threadIdx.x;
  if (i >= n_sets) return;
  fp12 f = fp12_one();
  if (b.status[i] == BLS_OK && pk_status[i] == BLS_OK && !(b.flags[b.n + i] & SF_H_INF)) {
    g1a P = ld_g1a(b.pk_aff, b.n, i);
    g2a Q = ld_g2a(b.h_aff, b.n, i);
    f = miller_loop(P, Q);
  }
  st_fp12(b.f, b.n, i, f);
}

static inline dim3 grid_for(uint32_t n) { return dim3((n + WAVE - 1) / WAVE); }

void launch_miller_sets(const PipelineBuffers& b, uint32_t n, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_miller_sets, grid_for(n), dim3(WAVE), 0, s, b, n, (const int8_t*)(b.status + b.n));
}

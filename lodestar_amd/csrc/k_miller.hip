// A12 per-set Miller loops f_i = MillerLoop(r_i pk_i, H(m_i)), one lane per set, in two passes
// (pairing.hpp "Two-pass Miller loop"):
//   k_miller_lines: T walks the 68 steps over Q = H(m_i); each step's Q-only line (l0, c1, c4) goes to HBM,
//                   SoA limb-major (step s, word w of set i at lines[(s * W_LINE + w) * n + i]: coalesced);
//   k_miller_acc:   f = prod_s line_s(P) with the squarings, from the stored lines; writes conj(f).
// Line traffic is 68 x 84 words = 22.8 KB per set each way (HBM-cheap next to ~6,700 Montgomery products).
#include "k_common.hpp"

#define W_LINE (3 * 2 * W_FP)

__device__ __forceinline__ bool miller_set_active(const PipelineBuffers& b, uint32_t i, const int8_t* pk_status) {
  return b.status[i] == BLS_OK && pk_status[i] == BLS_OK && !(b.flags[b.n + i] & SF_H_INF);
}

STAGE_KERNEL void k_miller_lines(PipelineBuffers b, uint32_t n_sets, const int8_t* pk_status) {
  uint32_t i = blockIdx.x * WAVE + threadIdx.x;
  if (i >= n_sets || !miller_set_active(b, i, pk_status)) return;
  const g2a Q = ld_g2a(b.h_aff, b.n, i);
  g2proj T;
  T.x = Q.x;
  T.y = Q.y;
  T.z = fp2_one();
  int bit = 62;
  bool add_next = false;
#pragma unroll 1
  for (int s = 0; s < MILLER_STEPS; s++) {
    line3 L;
    if (!add_next) {
      miller_dbl_line(T, L);
      add_next = (BLS_Z_ABS >> bit) & 1ull;
      bit--;
    } else {
      miller_add_line(T, Q, L);
      add_next = false;
    }
    uint32_t* o = b.lines + (size_t)s * W_LINE * b.n;
    st_fp2(o, b.n, i, 0, L.l0);
    st_fp2(o, b.n, i, 2 * W_FP, L.c1);
    st_fp2(o, b.n, i, 4 * W_FP, L.c4);
  }
}

STAGE_KERNEL void k_miller_acc(PipelineBuffers b, uint32_t n_sets, const int8_t* pk_status) {
  uint32_t i = blockIdx.x * WAVE + threadIdx.x;
  if (i >= n_sets) return;
  fp12 f = fp12_one();
  if (miller_set_active(b, i, pk_status)) {
    const g1a P = ld_g1a(b.pk_aff, b.n, i);
    int bit = 62;
    bool add_next = false;
#pragma unroll 1
    for (int s = 0; s < MILLER_STEPS; s++) {
      const uint32_t* o = b.lines + (size_t)s * W_LINE * b.n;
      line3 L;
      L.l0 = ld_fp2(o, b.n, i, 0);
      L.c1 = ld_fp2(o, b.n, i, 2 * W_FP);
      L.c4 = ld_fp2(o, b.n, i, 4 * W_FP);
      f = miller_acc_step(f, s, add_next, L, P.x, P.y);
      if (!add_next) {
        add_next = (BLS_Z_ABS >> bit) & 1ull;
        bit--;
      } else {
        add_next = false;
      }
    }
    f = fp12_conj(f);
  }
  st_fp12(b.f, b.n, i, f);
}

static inline dim3 grid_for(uint32_t n) { return dim3((n + WAVE - 1) / WAVE); }

void launch_miller_sets(const PipelineBuffers& b, uint32_t n, hipStream_t s) {
  if (!n) return;
  const int8_t* pk_status = (const int8_t*)(b.status + b.n);
  hipLaunchKernelGGL(k_miller_lines, grid_for(n), dim3(WAVE), 0, s, b, n, pk_status);
  hipLaunchKernelGGL(k_miller_acc, grid_for(n), dim3(WAVE), 0, s, b, n, pk_status);
}

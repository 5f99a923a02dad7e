// A12 Miller loops in two passes (pairing.hpp "Two-pass Miller loop"):
//   k_miller_lines: one lane per DISTINCT message: T walks the 68 steps over Q = H(m); each step's Q-only
//                   line (l0, c1, c4) goes to HBM, SoA limb-major (step s, word w of message u at
//                   lines[(s * W_LINE + w) * nm + u]: coalesced).  Lines depend on H(m) only, so every set
//                   and unit signing the same root shares them;
//   k_miller_acc:   one lane per chunk of <= K pairings of one batch group: f = prod_s prod_items line_s(P)
//                   with shared squarings, from the stored lines; writes conj(f).  An item is either one set
//                   (P = r_i pk_i) or, with same-message merging, a unit: the included sets of one batch
//                   group that sign the same root (P = sum r_i pk_i; the pairing is bilinear, so
//                   prod_i e(r_i pk_i, H(m)) = e(sum_i r_i pk_i, H(m))).
// Line traffic is 68 x 84 words = 22.8 KB per message (HBM-cheap next to ~5,200 Montgomery products).
#include "k_common.hpp"
#include "gt_wave.hpp"

STAGE_KERNEL_W(BLSGPU_WPE_LINES) void k_miller_lines(PipelineBuffers b) {
  uint32_t u = blockIdx.x * WAVE + threadIdx.x;
  if (u >= b.n_umsg || (b.mflags[u] & MF_H_INF)) return;
  const g2a Q = ld_g2a(b.h_aff, b.nm, u);
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
    uint32_t* o = b.lines + (size_t)s * W_LINE * b.nm;
    st_fp2(o, b.nm, u, 0, L.l0);
    st_fp2(o, b.nm, u, 2 * W_FP, L.c1);
    st_fp2(o, b.nm, u, 4 * W_FP, L.c4);
  }
}

// One lane per chunk: f = prod over the chunk's items of f_{|z|,Q_item}(P_item), with ONE Fp12 squaring per
// doubling step for the whole chunk (the multi-pairing form of blst's miller_loop_n): K items cost
// 63 squarings + 68 K line multiplications instead of K (63 + 68).  UNITS: item u is pairing unit u
// (P = unit_p[u]); otherwise item i is a set (P = r_i pk_i, only if it enters the batch equation).
template <bool UNITS>
STAGE_KERNEL_W(BLSGPU_WPE_ACC) void k_miller_acc(PipelineBuffers b) {
  const uint32_t c = blockIdx.x * WAVE + threadIdx.x;
  if (c >= b.n_chunks) return;
  const uint32_t k0 = b.chunk_first[c], k1 = b.chunk_first[c + 1];
  fp12 f = fp12_one();
  int bit = 62;
  bool add_next = false;
#pragma unroll 1
  for (int s = 0; s < MILLER_STEPS; s++) {
    if (!add_next && s != 0) f = fp12_sqr(f);
    const uint32_t* o = b.lines + (size_t)s * W_LINE * b.nm;
#pragma unroll 1
    for (uint32_t k = k0; k < k1; k++) {
      const uint32_t i = b.chunk_items[k];
      uint32_t m;
      bool active;
      if (UNITS) {
        m = b.unit_msg[i];
        active = b.unit_ok[i] != 0;
      } else {
        m = b.msg_idx[i];
        active = b.include[i] != 0;
      }
      if (!active || (b.mflags[m] & MF_H_INF)) continue;
      const g1a P = ld_g1a(UNITS ? b.unit_p : b.pk_aff, b.n, i);
      line3 L;
      L.l0 = ld_fp2(o, b.nm, m, 0);
      L.c1 = ld_fp2(o, b.nm, m, 2 * W_FP);
      L.c4 = ld_fp2(o, b.nm, m, 4 * W_FP);
      f = fp12_mul_by_014(f, L.l0, fp2_mul_fp(L.c1, P.x), fp2_mul_fp(L.c4, P.y));
    }
    if (!add_next) {
      add_next = (BLS_Z_ABS >> bit) & 1ull;
      bit--;
    } else {
      add_next = false;
    }
  }
  st_fp12(b.f_chunk, b.n, c, fp12_conj(f));
}

// Small runs (latency): one 128-lane workgroup per pairing, the Miller loop as cooperative Fp12 arithmetic
// (gt_wave.hpp: lines computed on the fly, one Fp product per lane per step) -- the same value as
// k_miller_lines + k_miller_acc with one item per chunk, in ~1/6 of the time per pairing, at a fraction of the
// lanes' efficiency; the runtime uses it only when the run's pairings fit the chip (runtime.cpp kCoopMaxItems).
template <bool UNITS>
__global__ __launch_bounds__(GTW_MILLER_LANES) void k_miller_coop(PipelineBuffers b) {
  __shared__ GtwLds sh;
  const uint32_t c = blockIdx.x, t = threadIdx.x;
  if (c >= b.n_chunks) return;
  const uint32_t i = b.chunk_items[b.chunk_first[c]];  // one item per chunk
  uint32_t m;
  bool active;
  if (UNITS) {
    m = b.unit_msg[i];
    active = b.unit_ok[i] != 0;
  } else {
    m = b.msg_idx[i];
    active = b.include[i] != 0;
  }
  active = active && !(b.mflags[m] & MF_H_INF);  // uniform over the workgroup
  if (active) {
    if (t < 4) lds_st(sh.QA, (int)t, ld_fp(b.h_aff, b.nm, m, (int)t * W_FP));
    const g1a P = ld_g1a(UNITS ? b.unit_p : b.pk_aff, b.n, i);
    gtw_sync();
    gtw_miller_loop(sh.G, sh.QA, P.x, P.y, sh.TB, sh.L, sh.L1, sh.S, sh.S2, t);
  } else {
    gtw_set_one(sh.G, t);
  }
  gtw_sync();
  for (uint32_t w = t; w < W_FP12; w += GTW_MILLER_LANES) b.f_chunk[(size_t)w * b.n + c] = sh.G[gtw_lds_word(w)];
}

static inline dim3 grid_for(uint32_t n) { return dim3((n + WAVE - 1) / WAVE); }

void launch_miller_coop(const PipelineBuffers& b, bool units, hipStream_t s, bool exclusive) {
  if (!b.n_chunks) return;
  if (units)
    hipLaunchKernelGGL(k_miller_coop<true>, dim3(b.n_chunks), dim3(GTW_MILLER_LANES),
                       exclusive ? exclusive_cu_lds<k_miller_coop<true>>() : 0, s, b);
  else
    hipLaunchKernelGGL(k_miller_coop<false>, dim3(b.n_chunks), dim3(GTW_MILLER_LANES),
                       exclusive ? exclusive_cu_lds<k_miller_coop<false>>() : 0, s, b);
}

void launch_miller_lines(const PipelineBuffers& b, hipStream_t s) {
  if (b.n_umsg) hipLaunchKernelGGL(k_miller_lines, grid_for(b.n_umsg), dim3(WAVE), 0, s, b);
}
void launch_miller_acc(const PipelineBuffers& b, bool units, hipStream_t s) {
  if (!b.n_chunks) return;
  if (units)
    hipLaunchKernelGGL(k_miller_acc<true>, grid_for(b.n_chunks), dim3(WAVE), 0, s, b);
  else
    hipLaunchKernelGGL(k_miller_acc<false>, grid_for(b.n_chunks), dim3(WAVE), 0, s, b);
}

// A12 Miller loops in two passes (pairing.hpp "Two-pass Miller loop"):
//   k_miller_lines: one lane per DISTINCT message: T walks the 68 steps over Q = H(m); each step's Q-only
//                   line (l0, c1, c4) goes to HBM, SoA limb-major (step s, word w of message u at
//                   lines[(s * W_LINE + w) * nm + u]: coalesced).  Lines depend on H(m) only, so every set
//                   and unit signing the same root shares them;
//   k_miller_acc:   one lane per pairing unit: f = prod_s line_s(P) with the squarings, from the stored lines;
//                   writes conj(f).  A unit is either one set (P = r_i pk_i) or, with same-message merging,
//                   the included sets of one batch group that sign the same root (P = sum r_i pk_i): the
//                   pairing is bilinear, so prod_i e(r_i pk_i, H(m)) = e(sum_i r_i pk_i, H(m)).
// Line traffic is 68 x 84 words = 22.8 KB per message (HBM-cheap next to ~5,200 Montgomery products).
#include "k_common.hpp"

STAGE_KERNEL void k_miller_lines(PipelineBuffers b) {
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

// UNITS: lane u is pairing unit u (P = unit_p[u], f -> f_unit[u]).  Otherwise lane u is set
// i = set_list ? set_list[u] : u (P = pk_aff[i], f -> f_set[i]); a set outside the batch equation gets f = 1.
template <bool UNITS>
STAGE_KERNEL void k_miller_acc(PipelineBuffers b, uint32_t n, const uint32_t* set_list) {
  uint32_t u = blockIdx.x * WAVE + threadIdx.x;
  if (u >= n) return;
  uint32_t i, m;
  bool active;
  const uint32_t* psrc;
  if (UNITS) {
    i = u;
    m = b.unit_msg[u];
    active = b.unit_ok[u] != 0;
    psrc = b.unit_p;
  } else {
    i = set_list ? set_list[u] : u;
    m = b.msg_idx[i];
    active = b.include[i] != 0;
    psrc = b.pk_aff;
  }
  active = active && !(b.mflags[m] & MF_H_INF);
  fp12 f = fp12_one();
  if (active) {
    const g1a P = ld_g1a(psrc, b.n, i);
    int bit = 62;
    bool add_next = false;
#pragma unroll 1
    for (int s = 0; s < MILLER_STEPS; s++) {
      const uint32_t* o = b.lines + (size_t)s * W_LINE * b.nm;
      line3 L;
      L.l0 = ld_fp2(o, b.nm, m, 0);
      L.c1 = ld_fp2(o, b.nm, m, 2 * W_FP);
      L.c4 = ld_fp2(o, b.nm, m, 4 * W_FP);
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
  st_fp12(UNITS ? b.f_unit : b.f_set, b.n, i, f);
}

static inline dim3 grid_for(uint32_t n) { return dim3((n + WAVE - 1) / WAVE); }

void launch_miller_lines(const PipelineBuffers& b, hipStream_t s) {
  if (b.n_umsg) hipLaunchKernelGGL(k_miller_lines, grid_for(b.n_umsg), dim3(WAVE), 0, s, b);
}
void launch_miller_acc(const PipelineBuffers& b, bool units, uint32_t n, const uint32_t* set_list, hipStream_t s) {
  if (!n) return;
  if (units)
    hipLaunchKernelGGL(k_miller_acc<true>, grid_for(n), dim3(WAVE), 0, s, b, n, set_list);
  else
    hipLaunchKernelGGL(k_miller_acc<false>, grid_for(n), dim3(WAVE), 0, s, b, n, set_list);
}

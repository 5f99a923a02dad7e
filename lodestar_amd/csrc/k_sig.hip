// A8 Signature.fromBytes(.., validate=true) (decompress + psi subgroup check) and the r_i * sig_i scaling
// of the random linear combination (A9), one lane per signature set.
#include "k_common.hpp"

STAGE_KERNEL_W(BLSGPU_WPE_DEC) void k_sig_decode(PipelineBuffers b, uint32_t n_sets) {
  uint32_t i = blockIdx.x * WAVE + threadIdx.x;
  if (i >= n_sets) return;
  uint8_t raw[192];
  uint32_t len = b.sig_len[i];
  const uint8_t* src = b.sigs + (size_t)i * b.sig_stride;
  uint32_t cl = len == 96 || len == 192 ? len : 0;
  for (uint32_t k = 0; k < cl; k++) raw[k] = src[k];
  g2a p;
  bool inf = false;
  int st = sig_decode_point(raw, len, p, inf);
  if (st != BLS_OK || inf) {
    p.x = fp2_zero();
    p.y = fp2_zero();
  }
  st_g2a(b.sig_aff, b.n, i, p);
  // subgroup check with P re-read from the output buffer (curve.hpp jac_mul_zabs_ld: no P across the chain)
  if (st == BLS_OK && !inf && !g2_in_subgroup_ld([&] { return ld_g2a(b.sig_aff, b.n, opaque_u32(i)); })) {
    st = BLS_POINT_NOT_IN_GROUP;
    p.x = fp2_zero();
    p.y = fp2_zero();
    st_g2a(b.sig_aff, b.n, i, p);
  }
  b.flags[i] = inf ? SF_SIG_INF : 0;  // sig flags: flags[0, n)
  b.status[i] = (int8_t)st;
}

// r_i sig_i with the batch scalar word (0 = r = 1, CoreVerify); the signed-window table goes to b.scal_tab.
// The fallback's path for small jobs (runtime.cpp): a per-set scaling costs less than a bucket MSM per 1-3-set job.
STAGE_KERNEL void k_sig_scale(PipelineBuffers b, uint32_t n_sets, const uint32_t* list) {
  const uint32_t q = blockIdx.x * WAVE + threadIdx.x;
  if (q >= n_sets) return;
  const uint32_t i = list ? list[q] : q;
  g2j R = jac_infinity<fp2>();
  if (b.status[i] == BLS_OK && !(b.flags[i] & SF_SIG_INF)) {
    const g2a s = ld_g2a(b.sig_aff, b.n, i);
    const uint64_t w = b.scalars[i];
    R = (w == 0) ? jac_from_aff(s) : jac_mul_scalar_word(jac_from_aff(s), w, b.scal_tab, b.n, i);
  }
  st_g2j(b.rsig, b.n, i, R);
}

static inline dim3 grid_for(uint32_t n) { return dim3((n + WAVE - 1) / WAVE); }

void launch_sig_decode(const PipelineBuffers& b, uint32_t n, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_sig_decode, grid_for(n), dim3(WAVE), 0, s, b, n);
}
void launch_sig_scale(const PipelineBuffers& b, uint32_t n, hipStream_t s, const uint32_t* list) {
  if (n) hipLaunchKernelGGL(k_sig_scale, grid_for(n), dim3(WAVE), 0, s, b, n, list);
}

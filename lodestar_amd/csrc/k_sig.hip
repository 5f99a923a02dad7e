// A8 Signature.fromBytes(.., validate=true) (decompress + psi subgroup check) and the r_i * sig_i scaling
// of the random linear combination (A9), one lane per signature set.
#include "k_common.hpp"
#include "g2_coop.hpp"

// check_group == false: the subgroup check is left to k_sig_subgroup_coop (small runs) or k_sig_subgroup2 (lane
// pairs, BLSGPU_SIG_PAIRS); the decode alone then fits two waves per SIMD (WPE_DEC0)
#ifndef BLSGPU_SIG_PAIRS
#define BLSGPU_SIG_PAIRS 1
#endif
#ifndef BLSGPU_WPE_DEC0
#define BLSGPU_WPE_DEC0 2
#endif
#ifndef BLSGPU_WPE_SUB2
#define BLSGPU_WPE_SUB2 2
#endif
template <bool CHECK, int WPE>
__global__ __launch_bounds__(WAVE) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) void k_sig_decode(
    PipelineBuffers b, uint32_t n_sets) {
  const bool check_group = CHECK;
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
  if (check_group && st == BLS_OK && !inf &&
      !g2_in_subgroup_ld([&] { return ld_g2a(b.sig_aff, b.n, opaque_u32(i)); })) {
    st = BLS_POINT_NOT_IN_GROUP;
    p.x = fp2_zero();
    p.y = fp2_zero();
    st_g2a(b.sig_aff, b.n, i, p);
  }
  b.flags[i] = inf ? SF_SIG_INF : 0;  // sig flags: flags[0, n)
  b.status[i] = (int8_t)st;
}

// The subgroup check psi(P) == [z]P of the decoded signatures on lane pairs (fp2x.hpp): lane 2i + k holds coefficient
// k of every Fp2 coordinate of signature i's chain -- half a point per lane, two waves per SIMD.  The affine P is
// re-read from the decode's output at each of the chain's mixed additions (curve.hpp jac_mul_zabs_lda).  A failing
// signature becomes POINT_NOT_IN_GROUP with a zero point, as in k_sig_decode.
STAGE_KERNEL_W(BLSGPU_WPE_SUB2) void k_sig_subgroup2(PipelineBuffers b, uint32_t n_sets) {
  const uint32_t q = blockIdx.x * WAVE + threadIdx.x, i = q >> 1, k = q & 1;
  if (i >= n_sets || b.status[i] != BLS_OK || (b.flags[i] & SF_SIG_INF)) return;  // per pair
  auto ldP = [&] {
    const uint32_t ii = opaque_u32(i);
    aff<fp2x> a;
    a.x.v = ld_fp(b.sig_aff, b.n, ii, (int)(k * W_FP));
    a.y.v = ld_fp(b.sig_aff, b.n, ii, (int)((2 + k) * W_FP));
    return a;
  };
  const g2jx zP = jac_neg(jac_mul_zabs_lda<fp2x>(ldP));
  if (!jac_eq(g2_psi(jac_from_aff(ldP())), zP)) {
    st_fp(b.sig_aff, b.n, i, (int)(k * W_FP), fp_zero());
    st_fp(b.sig_aff, b.n, i, (int)((2 + k) * W_FP), fp_zero());
    if (k == 0) b.status[i] = (int8_t)BLS_POINT_NOT_IN_GROUP;
  }
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

// The subgroup check psi(P) == [z]P of the decoded signatures for small runs, latency first: one 16-lane group per
// signature (g2_coop.hpp), the [|z|] chain as cooperative doublings, the additions and the comparison on the group's
// lane 0.  A failing signature becomes POINT_NOT_IN_GROUP with a zero point, as in k_sig_decode.
#define SG_GROUPS (WAVE / G2C_LANES)
__global__ __launch_bounds__(WAVE) void k_sig_subgroup_coop(PipelineBuffers b, uint32_t n_sets) {
  __shared__ uint32_t lds[SG_GROUPS * G2C_WORDS];
  const uint32_t tg = threadIdx.x % G2C_LANES, grp = threadIdx.x / G2C_LANES;
  const uint32_t i = blockIdx.x * SG_GROUPS + grp;
  uint32_t* g = lds + grp * G2C_WORDS;
  const bool on = i < n_sets && b.status[i] == BLS_OK && !(b.flags[i] & SF_SIG_INF);
  if (tg == 0 && on) g2c_st_point(g, jac_from_aff(ld_g2a(b.sig_aff, b.n, i)));
  g2c_sync();
  g2c_mul_zabs(g, tg, on, [&] { return jac_from_aff(ld_g2a(b.sig_aff, b.n, opaque_u32(i))); });
  if (tg == 0 && on) {
    const g2j zP = jac_neg(g2c_ld_point(g));
    if (!jac_eq(g2_psi(jac_from_aff(ld_g2a(b.sig_aff, b.n, i))), zP)) {
      g2a z;
      z.x = fp2_zero();
      z.y = fp2_zero();
      st_g2a(b.sig_aff, b.n, i, z);
      b.status[i] = (int8_t)BLS_POINT_NOT_IN_GROUP;
    }
  }
}

// the speculative MSM's mask (runtime.cpp): the sets whose signature decoded
__global__ __launch_bounds__(WAVE) void k_spec_mask(PipelineBuffers b, uint32_t n_sets, uint8_t* spec) {
  const uint32_t i = blockIdx.x * WAVE + threadIdx.x;
  if (i < n_sets) spec[i] = b.status[i] == BLS_OK ? 1 : 0;
}

static inline dim3 grid_for(uint32_t n) { return dim3((n + WAVE - 1) / WAVE); }

void launch_spec_mask(const PipelineBuffers& b, uint32_t n, uint8_t* spec, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_spec_mask, grid_for(n), dim3(WAVE), 0, s, b, n, spec);
}

void launch_sig_decode(const PipelineBuffers& b, uint32_t n, hipStream_t s, bool coop, hipEvent_t decoded,
                       bool exclusive) {
  if (!n) return;
  if (coop || BLSGPU_SIG_PAIRS)
    hipLaunchKernelGGL((k_sig_decode<false, BLSGPU_WPE_DEC0>), grid_for(n), dim3(WAVE), 0, s, b, n);
  else
    hipLaunchKernelGGL((k_sig_decode<true, BLSGPU_WPE_DEC>), grid_for(n), dim3(WAVE), 0, s, b, n);
  if (decoded) (void)hipEventRecord(decoded, s);
  if (!coop) {
    if (BLSGPU_SIG_PAIRS) hipLaunchKernelGGL(k_sig_subgroup2, grid_for(2 * n), dim3(WAVE), 0, s, b, n);
  } else
    hipLaunchKernelGGL(k_sig_subgroup_coop, dim3((n + SG_GROUPS - 1) / SG_GROUPS), dim3(WAVE),
                       BLSGPU_EXCLUSIVE_SMALL && exclusive ? exclusive_cu_lds<k_sig_subgroup_coop>() : 0, s, b, n);
}
void launch_sig_scale(const PipelineBuffers& b, uint32_t n, hipStream_t s, const uint32_t* list) {
  if (n) hipLaunchKernelGGL(k_sig_scale, grid_for(n), dim3(WAVE), 0, s, b, n, list);
}

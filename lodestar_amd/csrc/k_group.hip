// Batch-group tail of the random-linear-combination check (A7/A9), and the per-job error mask (A13).
//
// A batch group is a contiguous range of clean jobs checked with ONE final exponentiation:
//   prod_i e(r_i pk_i, H(m_i)) * e(-g1, sum_i r_i sig_i) == 1
// The per-set Miller loops f_i were computed by k_miller_sets; here
//   k_group_reduce   one wave per group: S = sum r_i sig_i (G2) and F = prod f_i (Fp12), each lane a strided
//                    partial, then a 6-level LDS tree (64 -> 1)
//   k_group_check    one lane per group: FinalExp(F * MillerLoop(-g1, S)) == 1
// The same two kernels re-check the sub-ranges of a failed group when the host bisects it
// (runtime.cpp), so the fallback costs one Miller loop + final exponentiation per tested sub-range.
#include "k_common.hpp"

// Lane per job: first error of the job, pubkeys before signatures (the reference deserializes pubkeys
// first, worker.ts:39 / maybeBatch.ts:23), and the include mask of its sets.
__global__ __launch_bounds__(WAVE) void k_job_mask(PipelineBuffers b) {
  uint32_t j = blockIdx.x * WAVE + threadIdx.x;
  if (j >= b.n_jobs) return;
  const uint32_t a = b.job_first_set[j], e = b.job_first_set[j + 1];
  const int8_t* pk_st = b.status + b.n;
  int err = 0;
  for (uint32_t i = a; i < e && !err; i++) err = pk_st[i];
  for (uint32_t i = a; i < e && !err; i++) err = b.status[i];
  if (a == e) err = BLS_EMPTY_SET;
  b.job_err[j] = (int8_t)err;
  for (uint32_t i = a; i < e; i++) b.include[i] = err == 0 ? 1 : 0;
}

__global__ __launch_bounds__(WAVE) void k_group_reduce(PipelineBuffers b, const uint32_t* ranges, uint32_t ng,
                                                       uint32_t* S_out, uint32_t* F_out) {
  __shared__ uint32_t red[WAVE * W_FP12];
  const uint32_t g = blockIdx.x, lane = threadIdx.x;
  if (g >= ng) return;
  const uint32_t first = ranges[2 * g], last = ranges[2 * g + 1];
  // ---- S = sum r_i sig_i
  g2j S = jac_infinity<fp2>();
  for (uint32_t i = first + lane; i < last; i += WAVE)
    if (b.include[i]) S = jac_add(S, ld_g2j(b.rsig, b.n, i));
#pragma unroll 1
  for (int s = WAVE / 2; s >= 1; s >>= 1) {
    if (lane >= (uint32_t)s && lane < (uint32_t)(2 * s)) st_g2j(red, WAVE, lane - s, S);
    __syncthreads();
    if (lane < (uint32_t)s) S = jac_add(S, ld_g2j(red, WAVE, lane));
    __syncthreads();
  }
  if (lane == 0) st_g2j(S_out, ng, g, S);
  // ---- F = prod f_i
  fp12 F = fp12_one();
  bool any = false;
  for (uint32_t i = first + lane; i < last; i += WAVE)
    if (b.include[i]) {
      F = any ? fp12_mul(F, ld_fp12(b.f, b.n, i)) : ld_fp12(b.f, b.n, i);
      any = true;
    }
#pragma unroll 1
  for (int s = WAVE / 2; s >= 1; s >>= 1) {
    if (lane >= (uint32_t)s && lane < (uint32_t)(2 * s)) st_fp12(red, WAVE, lane - s, F);
    __syncthreads();
    if (lane < (uint32_t)s) F = fp12_mul(F, ld_fp12(red, WAVE, lane));
    __syncthreads();
  }
  if (lane == 0) st_fp12(F_out, ng, g, F);
}

__global__ __launch_bounds__(WAVE) void k_group_check(const uint32_t* S_in, const uint32_t* F_in, uint32_t ng,
                                                      uint8_t* ok) {
  const uint32_t g = blockIdx.x * WAVE + threadIdx.x;
  if (g >= ng) return;
  fp12 f = ld_fp12(F_in, ng, g);
  g2a Sa;
  if (jac_to_aff(ld_g2j(S_in, ng, g), Sa)) {
    g1a ng1;
    ng1.x = G1_GEN_X;
    ng1.y = G1_NEG_GEN_Y;
    f = fp12_mul(f, miller_loop(ng1, Sa));
  }
  ok[g] = fp12_is_one(final_exponentiation(f)) ? 1 : 0;
}

static inline dim3 grid_for(uint32_t n) { return dim3((n + WAVE - 1) / WAVE); }

void launch_job_mask(const PipelineBuffers& b, hipStream_t s) {
  if (b.n_jobs) hipLaunchKernelGGL(k_job_mask, grid_for(b.n_jobs), dim3(WAVE), 0, s, b);
}
void launch_group_reduce(const PipelineBuffers& b, const uint32_t* ranges, uint32_t ng, uint32_t* S, uint32_t* F,
                         hipStream_t s) {
  if (ng) hipLaunchKernelGGL(k_group_reduce, dim3(ng), dim3(WAVE), 0, s, b, ranges, ng, S, F);
}
void launch_group_check(const uint32_t* S, const uint32_t* F, uint32_t ng, uint8_t* ok, hipStream_t s) {
  if (ng) hipLaunchKernelGGL(k_group_check, grid_for(ng), dim3(WAVE), 0, s, S, F, ng, ok);
}

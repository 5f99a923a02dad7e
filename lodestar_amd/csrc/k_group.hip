// Batch-group tail of the random-linear-combination check (A7/A9), and the per-job error mask (A13).
//
// A batch group is a contiguous range of clean jobs checked with ONE final exponentiation:
//   prod_i e(r_i pk_i, H(m_i)) * e(-g1, sum_i r_i sig_i) == 1
// The Miller values (chunks of sets or same-message units) were computed by k_miller_acc; here
//   k_group_reduce   one wave per group: F = prod f (Fp12), each lane a strided partial, then a 6-level LDS
//                    tree (64 -> 1); S = sum r_i sig_i comes from the bucket MSM (k_msm.hip)
//   k_group_check    one 128-lane workgroup per group: FinalExp(F * MillerLoop(-g1, S)) == 1, as
//                    workgroup-cooperative Fp12 arithmetic (gt_wave.hpp)
// The same two kernels re-check the sub-ranges of a failed group when the host bisects it
// (runtime.cpp), so the fallback costs one Miller loop + final exponentiation per tested sub-range.
#include "k_common.hpp"
#include "gt_wave.hpp"
#include "gt6.hpp"

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

__global__ __launch_bounds__(WAVE) void k_group_reduce(PipelineBuffers b, const uint32_t* f_ranges, uint32_t ng,
                                                       uint32_t* F_out) {
  __shared__ uint32_t red[WAVE * W_FP12];
  const uint32_t g = blockIdx.x, lane = threadIdx.x;
  if (g >= ng) return;
  // ---- F = prod of the group's Miller chunks
  const uint32_t first = f_ranges[2 * g], last = f_ranges[2 * g + 1];
  fp12 F = fp12_one();
  bool any = false;
  for (uint32_t i = first + lane; i < last; i += WAVE) {
    F = any ? fp12_mul(F, ld_fp12(b.f_chunk, b.n, i)) : ld_fp12(b.f_chunk, b.n, i);
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

// ---- F_g as a product tree (the batch pass) ---------------------------------------------------------------
// k_group_reduce above multiplies a group's chunks one wave per group: ~log2(chunks) + chunks / 64 lane-serial Fp12
// products deep (2.25 ms of a 16k call's critical path, 0.8 ms of a 128-set call's).  The tree form:
//   k_f_runs    lane per run of K consecutive chunks of a group (large runs only): their product into the run's first
//   k_f_pairs   one 128-lane workgroup per pair (dst, src) of one tree level: f[dst] *= f[src] as a cooperative
//               Fp12 product (gt_wave.hpp gtw_mul, ~5 us); the host plans the levels (runtime.cpp plan_f_tree)
//   k_f_gather  lane per (group, word): F_g = the group's first chunk (one for a group without chunks)
STAGE_KERNEL_W(BLSGPU_WPE_GRP) void k_f_runs(PipelineBuffers b, const uint32_t* runs, uint32_t n_runs) {
  const uint32_t q = blockIdx.x * WAVE + threadIdx.x;
  if (q >= n_runs) return;
  const uint32_t a = runs[2 * q], e = runs[2 * q + 1];
  fp12 F = ld_fp12(b.f_chunk, b.n, a);
#pragma unroll 1
  for (uint32_t i = a + 1; i < e; i++) F = fp12_mul(F, ld_fp12(b.f_chunk, b.n, i));
  st_fp12(b.f_chunk, b.n, a, F);
}

__global__ __launch_bounds__(GTW_LANES) void k_f_pairs(PipelineBuffers b, const uint32_t* pairs) {
  __shared__ uint32_t A[GTW_FP12], B[GTW_FP12], S[108 * BLS_NL];
  const uint32_t t = threadIdx.x, i = pairs[2 * blockIdx.x], j = pairs[2 * blockIdx.x + 1];
  for (uint32_t w = t; w < W_FP12; w += GTW_LANES) {
    A[gtw_lds_word(w)] = b.f_chunk[(size_t)w * b.n + i];
    B[gtw_lds_word(w)] = b.f_chunk[(size_t)w * b.n + j];
  }
  gtw_sync();
  gtw_mul<false>(A, A, B, S, t);
  for (uint32_t w = t; w < W_FP12; w += GTW_LANES) b.f_chunk[(size_t)w * b.n + i] = A[gtw_lds_word(w)];
}

STAGE_KERNEL void k_f_gather(PipelineBuffers b, const uint32_t* f_ranges, uint32_t ng, uint32_t* F_out) {
  const uint32_t q = blockIdx.x * WAVE + threadIdx.x;
  if (q >= ng * W_FP12) return;
  const uint32_t g = q % ng, w = q / ng, a = f_ranges[2 * g], e = f_ranges[2 * g + 1];
  F_out[q] = a < e ? b.f_chunk[(size_t)w * b.n + a] : (w < BLS_NL ? FP_ONE.l[w] : 0u);
}

// One 128-lane workgroup per group: the Miller loop and the final exponentiation run as cooperative Fp12
// arithmetic (gt_wave.hpp), one Fp product per lane per step.
//   G_in == nullptr: FinalExp(F * MillerLoop(-g1, S)) == 1 (the fallback's per-job / sub-group checks);
//   G_in != nullptr: FinalExp(F * G) == 1 with G = MillerLoop(-g1, S) from k_group_sig_miller, which the batch
//                    pass runs right after the MSM, beside the message branch (off the call's critical path).
// F / G in HBM: SoA tower layout (Fp2 slots c0.c0, c0.c1, c0.c2, c1.c0, c1.c1, c1.c2); in LDS: the w-basis.
// lane 0: S -> affine in QA; returns (through LDS) whether S is finite
__device__ __forceinline__ void gtw_load_S(GtwLds& sh, const uint32_t* S_in, uint32_t ng, uint32_t g, uint32_t t) {
  if (t == 0) {
    g2a Sa;
    const bool fin = jac_to_aff(ld_g2j(S_in, ng, g), Sa);
    if (fin) {
      lds_st(sh.QA, 0, Sa.x.c0);
      lds_st(sh.QA, 1, Sa.x.c1);
      lds_st(sh.QA, 2, Sa.y.c0);
      lds_st(sh.QA, 3, Sa.y.c1);
    }
    sh.flag = fin ? 1u : 0u;
  }
}

__global__ __launch_bounds__(GTW_MILLER_LANES) void k_group_sig_miller(const uint32_t* S_in, uint32_t ng, uint32_t* G_out) {
  __shared__ GtwLds sh;
  const uint32_t g = blockIdx.x, t = threadIdx.x;
  gtw_load_S(sh, S_in, ng, g, t);
  gtw_sync();
  if (sh.flag)
    gtw_miller_loop(sh.G, sh.QA, G1_GEN_X, G1_NEG_GEN_Y, sh.TB, sh.L, sh.L1, sh.S, sh.S2, t);
  else
    gtw_set_one(sh.G, t);
  gtw_sync();
  for (uint32_t w = t; w < W_FP12; w += GTW_MILLER_LANES) G_out[(size_t)w * ng + g] = sh.G[gtw_lds_word(w)];
}

// The same G = MillerLoop(-g1, S) on one lane per group (pairing.hpp miller_loop: conj(f), the layout above) for
// merged runs, where a three-wave cooperative workgroup waits for three free SIMDs of one CU (~20 ms per launch in the
// driver's trace, on the run's critical path) while single waves take any free SIMD.
STAGE_KERNEL_W(BLSGPU_WPE_GRP) void k_group_sig_miller_lane(const uint32_t* S_in, uint32_t ng, uint32_t* G_out) {
  const uint32_t g = blockIdx.x * WAVE + threadIdx.x;
  if (g >= ng) return;
  g2a Sa;
  g1a P;
  P.x = G1_GEN_X;
  P.y = G1_NEG_GEN_Y;
  const fp12 G = jac_to_aff(ld_g2j(S_in, ng, g), Sa) ? miller_loop(P, Sa) : fp12_one();
  st_fp12(G_out, ng, g, G);
}

// Lines of S for the fallback's six-lane checks: lane per entry sel[q] (all ng when sel is null): S -> affine, its 68
// Miller lines to column sel[q] of `lines` (stride ng); flags[sel[q]] = 1 when S is the identity (no lines).
STAGE_KERNEL_W(BLSGPU_WPE_LINES) void k_check_lines(const uint32_t* S_in, uint32_t ng, const uint32_t* sel, uint32_t n,
                                                   uint32_t* lines, uint8_t* flags) {
  const uint32_t q = blockIdx.x * WAVE + threadIdx.x;
  if (q >= n) return;
  const uint32_t g = sel ? sel[q] : q;
  g2a Sa;
  const bool fin = jac_to_aff(ld_g2j(S_in, ng, g), Sa);
  flags[g] = fin ? 0 : 1;
  if (fin) miller_lines_store(Sa, lines, ng, g);
}

// the same for the entries sel[0 .. n) only (G columns sel[q]; the fallback's six-lane checks)
STAGE_KERNEL_W(BLSGPU_WPE_GRP) void k_group_sig_miller_lane_sel(const uint32_t* S_in, uint32_t ng, const uint32_t* sel,
                                                               uint32_t n, uint32_t* G_out) {
  const uint32_t q = blockIdx.x * WAVE + threadIdx.x;
  if (q >= n) return;
  const uint32_t g = sel ? sel[q] : q;
  g2a Sa;
  g1a P;
  P.x = G1_GEN_X;
  P.y = G1_NEG_GEN_Y;
  const fp12 G = jac_to_aff(ld_g2j(S_in, ng, g), Sa) ? miller_loop(P, Sa) : fp12_one();
  st_fp12(G_out, ng, g, G);
}

// MILLER: G_in is null, the kernel runs MillerLoop(-g1, S) itself (three waves, gtw_miller_loop); otherwise two
template <bool MILLER>
__global__ __launch_bounds__(MILLER ? GTW_MILLER_LANES : GTW_LANES) void k_group_check(
    const uint32_t* S_in, const uint32_t* F_in, uint32_t ng, const uint32_t* G_in, const uint32_t* sel, uint8_t* ok) {
  constexpr uint32_t NT = MILLER ? GTW_MILLER_LANES : GTW_LANES;
  __shared__ GtwLds sh;
  const uint32_t t = threadIdx.x;
  const uint32_t g = sel ? sel[blockIdx.x] : blockIdx.x;  // entry checked (S_in / F_in stride ng); verdict ok[blockIdx.x]
  for (uint32_t w = t; w < W_FP12; w += NT) {
    sh.F[gtw_lds_word(w)] = F_in[(size_t)w * ng + g];
    if (!MILLER) sh.G[gtw_lds_word(w)] = G_in[(size_t)w * ng + g];
  }
  if (MILLER) gtw_load_S(sh, S_in, ng, g, t);
  gtw_sync();
  if (!MILLER) {
    gtw_mul<false>(sh.F, sh.F, sh.G, sh.S, t);
  } else if (sh.flag) {
    gtw_miller_loop(sh.G, sh.QA, G1_GEN_X, G1_NEG_GEN_Y, sh.TB, sh.L, sh.L1, sh.S, sh.S2, t);
    gtw_mul<false>(sh.F, sh.F, sh.G, sh.S, t);
  }
  gtw_final_exp(sh.F, sh.W, sh.S, t);
  if (t == 0) ok[blockIdx.x] = fp12_is_one(gtw_to_reg(sh.F)) ? 1 : 0;
}

// The same check on ONE lane per entry (pairing.hpp miller_loop + final_exponentiation): ~64x the cooperative form's
// latency per check but a few percent of its chip time -- for the fallback of merged runs under load, where thousands
// of checks at once left the cooperative workgroups contending for SIMDs at ~1% of the VALU peak (r05 trace: 3,424
// checks in 36-46 ms) while one wave of lanes takes 64 checks on one SIMD.
STAGE_KERNEL_W(BLSGPU_WPE_GRP) void k_group_check_lane(const uint32_t* S_in, const uint32_t* F_in, uint32_t ng,
                                                      const uint32_t* sel, uint32_t n, uint8_t* ok) {
  const uint32_t q = blockIdx.x * WAVE + threadIdx.x;
  if (q >= n) return;
  const uint32_t g = sel ? sel[q] : q;
  fp12 F = ld_fp12(F_in, ng, g);
  g2a Sa;
  if (jac_to_aff(ld_g2j(S_in, ng, g), Sa)) {
    g1a P;
    P.x = G1_GEN_X;
    P.y = G1_NEG_GEN_Y;
    F = fp12_mul(F, miller_loop(P, Sa));
  }
  ok[q] = fp12_is_one(final_exponentiation(F)) ? 1 : 0;
}

// The fallback's checks on SIX lanes per check (gt6.hpp): FinalExp(F * G) == 1 with G = MillerLoop(-g1, S) computed
// beforehand (k_group_sig_miller_lane) -- the final exponentiation in ~1/6 of the one-lane time, ten checks per wave:
// for the dense-failure launches of merged runs under load, where a one-lane check's ~25 ms was the run's latency.
// MILLER: G = MillerLoop(-g1, S) on the same six lanes from S's stored lines (k_check_lines; flags[gi] set: S is the
// identity, G = 1), else G_in.
template <bool MILLER>
STAGE_KERNEL_W(BLSGPU_WPE_GRP) void k_group_check6(const uint32_t* F_in, const uint32_t* G_in, uint32_t ng,
                                                  const uint32_t* sel, uint32_t n, uint8_t* ok, const uint32_t* lines,
                                                  const uint8_t* flags) {
  const uint32_t lane = threadIdx.x, grp = lane / 6, k = lane % 6;
  const uint32_t q = blockIdx.x * ACC6_GROUPS + grp;
  if (grp >= ACC6_GROUPS || q >= n) return;  // whole groups leave together
  const uint32_t gi = sel ? sel[q] : q;
  const G6 g{(int)(grp * 6), k};
  const int w0 = ((k & 1) ? 3 : 0) * 2 * W_FP + (int)(k >> 1) * 2 * W_FP;
  const fp2 F = ld_fp2(F_in, ng, gi, w0);
  fp2 G;
  if (MILLER)
    G = flags[gi] ? (k == 0 ? fp2_one() : fp2_zero()) : g6_miller(lines, ng, gi, G1_GEN_X, G1_NEG_GEN_Y, g);
  else
    G = ld_fp2(G_in, ng, gi, w0);
  const bool one = g6_is_one(g6_final_exp(g6_mul(F, G, g), g), g);
  if (k == 0) ok[q] = one ? 1 : 0;
}

// Fallback sub-groups: S_out[r] = sum S_in[e], F_out[r] = prod F_in[e] over the entries e of range r
// (entries = per-job values, stride n_in; one wave per range, strided partials + LDS tree).
__global__ __launch_bounds__(WAVE) void k_range_combine(const uint32_t* S_in, const uint32_t* F_in, uint32_t n_in,
                                                        const uint32_t* ranges, uint32_t n_out, uint32_t* S_out,
                                                        uint32_t* F_out) {
  __shared__ uint32_t red[WAVE * (W_G2J + W_FP12)];
  const uint32_t r = blockIdx.x, lane = threadIdx.x;
  if (r >= n_out) return;
  const uint32_t first = ranges[2 * r], last = ranges[2 * r + 1];
  g2j S = jac_infinity<fp2>();
  fp12 F = fp12_one();
  for (uint32_t e = first + lane; e < last; e += WAVE) {
    S = jac_add(S, ld_g2j(S_in, n_in, e));
    F = fp12_mul(F, ld_fp12(F_in, n_in, e));
  }
#pragma unroll 1
  for (int h = WAVE / 2; h >= 1; h >>= 1) {
    if (lane >= (uint32_t)h && lane < (uint32_t)(2 * h)) {
      st_g2j(red, WAVE, lane - h, S);
      st_fp12(red + WAVE * W_G2J, WAVE, lane - h, F);
    }
    __syncthreads();
    if (lane < (uint32_t)h) {
      S = jac_add(S, ld_g2j(red, WAVE, lane));
      F = fp12_mul(F, ld_fp12(red + WAVE * W_G2J, WAVE, lane));
    }
    __syncthreads();
  }
  if (lane == 0) {
    st_g2j(S_out, n_out, r, S);
    st_fp12(F_out, n_out, r, F);
  }
}

// ---- lane-per-item forms of the fallback's reductions (many tiny ranges: one lane each) ----------------------

// lane per range: S = sum of the range's included r_i sig_i (b.rsig), F = prod of its Miller chunks (b.f_chunk)
STAGE_KERNEL_W(BLSGPU_WPE_GRP) void k_group_reduce_lane(PipelineBuffers b, const uint32_t* set_ranges, const uint32_t* f_ranges,
                                      uint32_t ng, uint32_t* S_out, uint32_t* F_out) {
  const uint32_t g = blockIdx.x * WAVE + threadIdx.x;
  if (g >= ng) return;
  g2j S = jac_infinity<fp2>();
  for (uint32_t i = set_ranges[2 * g]; i < set_ranges[2 * g + 1]; i++)
    if (b.include[i]) S = jac_add(S, ld_g2j(b.rsig, b.n, i));
  fp12 F = fp12_one();
  for (uint32_t c = f_ranges[2 * g]; c < f_ranges[2 * g + 1]; c++) F = fp12_mul(F, ld_fp12(b.f_chunk, b.n, c));
  st_g2j(S_out, ng, g, S);
  st_fp12(F_out, ng, g, F);
}

// lane per sub-group: S_out[r] = sum, F_out[r] = prod of entries ranges[2r] .. ranges[2r+1] (stride n_in)
STAGE_KERNEL_W(BLSGPU_WPE_GRP) void k_range_combine_lane(const uint32_t* S_in, const uint32_t* F_in, uint32_t n_in, const uint32_t* ranges,
                                       uint32_t n_out, uint32_t* S_out, uint32_t* F_out) {
  const uint32_t r = blockIdx.x * WAVE + threadIdx.x;
  if (r >= n_out) return;
  g2j S = jac_infinity<fp2>();
  fp12 F = fp12_one();
  for (uint32_t e = ranges[2 * r]; e < ranges[2 * r + 1]; e++) {
    S = jac_add(S, ld_g2j(S_in, n_in, e));
    F = fp12_mul(F, ld_fp12(F_in, n_in, e));
  }
  st_g2j(S_out, n_out, r, S);
  st_fp12(F_out, n_out, r, F);
}

static inline dim3 grid_for(uint32_t n) { return dim3((n + WAVE - 1) / WAVE); }

// word copy on the caller's stream (the batch pass's per-set Miller values kept aside for the fallback, runtime keep_f)
__global__ __launch_bounds__(256) void k_copy_words(uint32_t* __restrict__ dst, const uint32_t* __restrict__ src,
                                                    size_t n) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) dst[i] = src[i];
}
void launch_copy_words(uint32_t* dst, const uint32_t* src, size_t n, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_copy_words, dim3((unsigned)std::min<size_t>((n + 255) / 256, 8192)), dim3(256), 0, s, dst, src, n);
}

void launch_group_reduce_lane(const PipelineBuffers& b, const uint32_t* set_ranges, const uint32_t* f_ranges,
                              uint32_t ng, uint32_t* S, uint32_t* F, hipStream_t s) {
  if (ng) hipLaunchKernelGGL(k_group_reduce_lane, grid_for(ng), dim3(WAVE), 0, s, b, set_ranges, f_ranges, ng, S, F);
}
void launch_range_combine_lane(const uint32_t* S_in, const uint32_t* F_in, uint32_t n_in, const uint32_t* ranges,
                               uint32_t n_out, uint32_t* S_out, uint32_t* F_out, hipStream_t s) {
  if (n_out)
    hipLaunchKernelGGL(k_range_combine_lane, grid_for(n_out), dim3(WAVE), 0, s, S_in, F_in, n_in, ranges, n_out, S_out,
                       F_out);
}

void launch_job_mask(const PipelineBuffers& b, hipStream_t s) {
  if (b.n_jobs) hipLaunchKernelGGL(k_job_mask, grid_for(b.n_jobs), dim3(WAVE), 0, s, b);
}
void launch_group_reduce(const PipelineBuffers& b, const uint32_t* f_ranges, uint32_t ng, uint32_t* F, hipStream_t s) {
  if (ng) hipLaunchKernelGGL(k_group_reduce, dim3(ng), dim3(WAVE), 0, s, b, f_ranges, ng, F);
}
void launch_group_tree(const PipelineBuffers& b, const uint32_t* f_ranges, uint32_t ng, const uint32_t* runs,
                       uint32_t n_runs, const uint32_t* pairs, const std::vector<uint32_t>& level_end, uint32_t* F,
                       hipStream_t s) {
  if (!ng) return;
  if (n_runs) hipLaunchKernelGGL(k_f_runs, grid_for(n_runs), dim3(WAVE), 0, s, b, runs, n_runs);
  uint32_t p0 = 0;
  for (const uint32_t p1 : level_end) {
    if (p1 > p0) hipLaunchKernelGGL(k_f_pairs, dim3(p1 - p0), dim3(GTW_LANES), 0, s, b, pairs + 2 * (size_t)p0);
    p0 = p1;
  }
  hipLaunchKernelGGL(k_f_gather, grid_for(ng * W_FP12), dim3(WAVE), 0, s, b, f_ranges, ng, F);
}
void launch_group_sig_miller_sel(const uint32_t* S, uint32_t ng, const uint32_t* sel, uint32_t n_sel, uint32_t* G,
                                 hipStream_t s) {
  const uint32_t n = sel ? n_sel : ng;
  if (n) hipLaunchKernelGGL(k_group_sig_miller_lane_sel, grid_for(n), dim3(WAVE), 0, s, S, ng, sel, n, G);
}
void launch_group_check6(const uint32_t* F, const uint32_t* G, uint32_t ng, uint8_t* ok, hipStream_t s,
                         const uint32_t* sel, uint32_t n_sel) {
  const uint32_t n = sel ? n_sel : ng;
  if (n)
    hipLaunchKernelGGL(k_group_check6<false>, dim3((n + ACC6_GROUPS - 1) / ACC6_GROUPS), dim3(WAVE), 0, s, F, G, ng,
                       sel, n, ok, nullptr, nullptr);
}
void launch_check6_miller(const uint32_t* S, const uint32_t* F, uint32_t ng, uint8_t* ok, hipStream_t s,
                          const uint32_t* sel, uint32_t n_sel, uint32_t* lines, uint8_t* flags) {
  const uint32_t n = sel ? n_sel : ng;
  if (!n) return;
  hipLaunchKernelGGL(k_check_lines, grid_for(n), dim3(WAVE), 0, s, S, ng, sel, n, lines, flags);
  hipLaunchKernelGGL(k_group_check6<true>, dim3((n + ACC6_GROUPS - 1) / ACC6_GROUPS), dim3(WAVE), 0, s, F, nullptr, ng,
                     sel, n, ok, lines, flags);
}
void launch_group_check(const uint32_t* S, const uint32_t* F, uint32_t ng, uint8_t* ok, hipStream_t s,
                        const uint32_t* sel, uint32_t n_sel, const uint32_t* G, bool exclusive, bool lane) {
  const uint32_t n = sel ? n_sel : ng;
  if (!n) return;
  if (lane && !G)
    hipLaunchKernelGGL(k_group_check_lane, grid_for(n), dim3(WAVE), 0, s, S, F, ng, sel, n, ok);
  else if (G)
    hipLaunchKernelGGL(k_group_check<false>, dim3(n), dim3(GTW_LANES),
                       exclusive ? exclusive_cu_lds<k_group_check<false>>() : 0, s, S, F, ng, G, sel, ok);
  else
    hipLaunchKernelGGL(k_group_check<true>, dim3(n), dim3(GTW_MILLER_LANES),
                       exclusive ? exclusive_cu_lds<k_group_check<true>>() : 0, s, S, F, ng, G, sel, ok);
}
void launch_group_sig_miller(const uint32_t* S, uint32_t ng, uint32_t* G, hipStream_t s, bool exclusive, bool lane) {
  if (ng && lane)
    hipLaunchKernelGGL(k_group_sig_miller_lane, grid_for(ng), dim3(WAVE), 0, s, S, ng, G);
  else if (ng)
    hipLaunchKernelGGL(k_group_sig_miller, dim3(ng), dim3(GTW_MILLER_LANES),
                       exclusive ? exclusive_cu_lds<k_group_sig_miller>() : 0,
                       s, S, ng, G);
}
void launch_range_combine(const uint32_t* S_in, const uint32_t* F_in, uint32_t n_in, const uint32_t* ranges,
                          uint32_t n_out, uint32_t* S_out, uint32_t* F_out, hipStream_t s) {
  if (n_out)
    hipLaunchKernelGGL(k_range_combine, dim3(n_out), dim3(WAVE), 0, s, S_in, F_in, n_in, ranges, n_out, S_out, F_out);
}

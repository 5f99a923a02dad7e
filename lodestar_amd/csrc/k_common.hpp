// Shared device helpers of the verification kernels: SoA limb-major loads/stores (element i, word w at
// base[w * stride + i], so the 64 lanes of a wave touch 64 consecutive words per limb -- coalesced) and
// the small scalar-multiplication loops.  Included by every k_*.hip translation unit.
#pragma once
#include <atomic>

#include "kernels.h"
#include "ops.hpp"
#include "fp2x.hpp"

#define WAVE 64
#if defined(__HIP_DEVICE_COMPILE__) && !BLS_INLINE_PRODUCTS && !BLS_FP2_CLASSIC
// fp2_mul's LDS argument slot is indexed by threadIdx.x: every launch shape of the kernels stays within it
// (BLSGPU_DEBUG=1 builds also assert it at run time, tower.hpp)
static_assert(WAVE <= BLS_FP2_LDS_LANES, "fp2_mul LDS slot");
static_assert(2 * WAVE <= BLS_FP2_LDS_LANES, "128-lane kernels (gt_wave.hpp, k_msm_bucket) and fp2_mul LDS slot");
#endif

// Lane-per-set stage kernels.  BLSGPU_WPE is the number of waves per SIMD the register budget is sized for:
// 1 lets a kernel take the whole 512-entry VGPR+AGPR file (no spills, but one resident wave per SIMD, so
// concurrent batches cannot share a SIMD); 2 halves the budget so two in-flight batches co-reside and hide
// each other's dependent-MAD latency, at the price of scratch spills.
#ifndef BLSGPU_WPE
#define BLSGPU_WPE 1
#endif
#define STAGE_KERNEL __global__ __launch_bounds__(WAVE) __attribute__((amdgpu_waves_per_eu(BLSGPU_WPE, BLSGPU_WPE)))
// Per-kernel register budgets (waves per SIMD), default BLSGPU_WPE: a kernel whose live state fits 256 registers
// with little spilling can take two waves per SIMD, so two waves hide each other's dependent-MAD latency.
#define STAGE_KERNEL_W(w) __global__ __launch_bounds__(WAVE) __attribute__((amdgpu_waves_per_eu(w, w)))
// k_pk_finish at two waves (256 registers, 368 B scratch): C2 within noise, C4 2.42M -> 2.16M (r05aa): one wave
#ifndef BLSGPU_WPE_PK
#define BLSGPU_WPE_PK BLSGPU_WPE
#endif
// k_hash_prep at two waves: C2 within noise, slightly lower (3.72M vs 3.77M, three rounds of 100 steps): one wave
#ifndef BLSGPU_WPE_HPREP
#define BLSGPU_WPE_HPREP 1
#endif
#ifndef BLSGPU_WPE_MSM
#define BLSGPU_WPE_MSM BLSGPU_WPE
#endif
#ifndef BLSGPU_WPE_LINES
#define BLSGPU_WPE_LINES BLSGPU_WPE
#endif
#ifndef BLSGPU_WPE_ACC
#define BLSGPU_WPE_ACC BLSGPU_WPE
#endif
#ifndef BLSGPU_WPE_DEC
#define BLSGPU_WPE_DEC BLSGPU_WPE
#endif
#ifndef BLSGPU_WPE_HASH
#define BLSGPU_WPE_HASH BLSGPU_WPE
#endif
#ifndef BLSGPU_WPE_HMAP
#define BLSGPU_WPE_HMAP 2
#endif
#ifndef BLSGPU_WPE_GRP
#define BLSGPU_WPE_GRP BLSGPU_WPE
#endif

// x, hidden from the optimizer: an SoA load whose lane index goes through this is recomputed where it is issued.
// Inside a loop (the five additions of a [|z|] chain) the compiler otherwise hoists the point's 84 loop-invariant
// 64-bit addresses out of the loop and spills them to scratch around the product calls.
__device__ __forceinline__ uint32_t opaque_u32(uint32_t x) {
  asm volatile("" : "+v"(x));
  return x;
}

__device__ __forceinline__ fp ld_fp(const uint32_t* p, uint32_t n, uint32_t i, int w0) {
  fp r;
#pragma unroll
  for (int l = 0; l < BLS_NL; l++) r.l[l] = p[(size_t)(w0 + l) * n + i];
  return r;
}
__device__ __forceinline__ void st_fp(uint32_t* p, uint32_t n, uint32_t i, int w0, const fp& v) {
#pragma unroll
  for (int l = 0; l < BLS_NL; l++) p[(size_t)(w0 + l) * n + i] = v.l[l];
}
__device__ __forceinline__ fp2 ld_fp2(const uint32_t* p, uint32_t n, uint32_t i, int w0) {
  return fp2_make(ld_fp(p, n, i, w0), ld_fp(p, n, i, w0 + W_FP));
}
__device__ __forceinline__ void st_fp2(uint32_t* p, uint32_t n, uint32_t i, int w0, const fp2& v) {
  st_fp(p, n, i, w0, v.c0);
  st_fp(p, n, i, w0 + W_FP, v.c1);
}
__device__ __forceinline__ g2a ld_g2a(const uint32_t* p, uint32_t n, uint32_t i) {
  g2a r;
  r.x = ld_fp2(p, n, i, 0);
  r.y = ld_fp2(p, n, i, 2 * W_FP);
  return r;
}
__device__ __forceinline__ void st_g2a(uint32_t* p, uint32_t n, uint32_t i, const g2a& v) {
  st_fp2(p, n, i, 0, v.x);
  st_fp2(p, n, i, 2 * W_FP, v.y);
}
__device__ __forceinline__ g2j ld_g2j(const uint32_t* p, uint32_t n, uint32_t i) {
  g2j r;
  r.x = ld_fp2(p, n, i, 0);
  r.y = ld_fp2(p, n, i, 2 * W_FP);
  r.z = ld_fp2(p, n, i, 4 * W_FP);
  return r;
}
__device__ __forceinline__ void st_g2j(uint32_t* p, uint32_t n, uint32_t i, const g2j& v) {
  st_fp2(p, n, i, 0, v.x);
  st_fp2(p, n, i, 2 * W_FP, v.y);
  st_fp2(p, n, i, 4 * W_FP, v.z);
}
__device__ __forceinline__ g1a ld_g1a(const uint32_t* p, uint32_t n, uint32_t i) {
  g1a r;
  r.x = ld_fp(p, n, i, 0);
  r.y = ld_fp(p, n, i, W_FP);
  return r;
}
__device__ __forceinline__ void st_g1a(uint32_t* p, uint32_t n, uint32_t i, const g1a& v) {
  st_fp(p, n, i, 0, v.x);
  st_fp(p, n, i, W_FP, v.y);
}
__device__ __forceinline__ g1j ld_g1j(const uint32_t* p, uint32_t n, uint32_t i) {
  g1j r;
  r.x = ld_fp(p, n, i, 0);
  r.y = ld_fp(p, n, i, W_FP);
  r.z = ld_fp(p, n, i, 2 * W_FP);
  return r;
}
__device__ __forceinline__ void st_g1j(uint32_t* p, uint32_t n, uint32_t i, const g1j& v) {
  st_fp(p, n, i, 0, v.x);
  st_fp(p, n, i, W_FP, v.y);
  st_fp(p, n, i, 2 * W_FP, v.z);
}
__device__ __forceinline__ fp12 ld_fp12(const uint32_t* p, uint32_t n, uint32_t i) {
  fp12 f;
  f.c0.c0 = ld_fp2(p, n, i, 0);
  f.c0.c1 = ld_fp2(p, n, i, 2 * W_FP);
  f.c0.c2 = ld_fp2(p, n, i, 4 * W_FP);
  f.c1.c0 = ld_fp2(p, n, i, 6 * W_FP);
  f.c1.c1 = ld_fp2(p, n, i, 8 * W_FP);
  f.c1.c2 = ld_fp2(p, n, i, 10 * W_FP);
  return f;
}
__device__ __forceinline__ void st_fp12(uint32_t* p, uint32_t n, uint32_t i, const fp12& f) {
  st_fp2(p, n, i, 0, f.c0.c0);
  st_fp2(p, n, i, 2 * W_FP, f.c0.c1);
  st_fp2(p, n, i, 4 * W_FP, f.c0.c2);
  st_fp2(p, n, i, 6 * W_FP, f.c1.c0);
  st_fp2(p, n, i, 8 * W_FP, f.c1.c1);
  st_fp2(p, n, i, 10 * W_FP, f.c1.c2);
}
// lane pairs (fp2x.hpp): coefficient k of every Fp2 coordinate of SoA point i (c_k at words (2 c + k) W_FP ..)
__device__ __forceinline__ g2jx ld_g2jx(const uint32_t* p, uint32_t n, uint32_t i, uint32_t k) {
  g2jx r;
  r.x.v = ld_fp(p, n, i, (int)(k * W_FP));
  r.y.v = ld_fp(p, n, i, (int)((2 + k) * W_FP));
  r.z.v = ld_fp(p, n, i, (int)((4 + k) * W_FP));
  return r;
}
__device__ __forceinline__ void st_g2jx(uint32_t* p, uint32_t n, uint32_t i, uint32_t k, const g2jx& v) {
  st_fp(p, n, i, (int)(k * W_FP), v.x.v);
  st_fp(p, n, i, (int)((2 + k) * W_FP), v.y.v);
  st_fp(p, n, i, (int)((4 + k) * W_FP), v.z.v);
}
// lane-pair exchange (lane ^ 1) of register values: __shfl_xor, no LDS
BLS_INL fp fp_xlane(const fp& x) {
  fp r;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) r.l[i] = (uint32_t)__shfl_xor((int)x.l[i], 1);
  return r;
}
BLS_INL fp2 fp2_xlane(const fp2& x) { return fp2_make(fp_xlane(x.c0), fp_xlane(x.c1)); }
BLS_INL fp6 fp6_xlane(const fp6& x) { return fp6_make(fp2_xlane(x.c0), fp2_xlane(x.c1), fp2_xlane(x.c2)); }
// The 68 Miller lines of Q (affine, finite) in Q-only form (l0, c1, c4), step s of column u at
// lines[(s * W_LINE + w) * nm + u] (k_miller_lines: one column per distinct message; k_check_lines: per fallback check)
__device__ __forceinline__ void miller_lines_store(const g2a& Q, uint32_t* lines, uint32_t nm, uint32_t u) {
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
    uint32_t* o = lines + (size_t)s * W_LINE * nm;
    st_fp2(o, nm, u, 0, L.l0);
    st_fp2(o, nm, u, 2 * W_FP, L.c1);
    st_fp2(o, nm, u, 4 * W_FP, L.c4);
  }
}

// any-lane exchange of register values (ds_bpermute; the lane-group kernels k_miller_acc6 / gt6.hpp)
BLS_INL fp fp_shfl(const fp& x, int src) {
  fp r;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) r.l[i] = (uint32_t)__shfl((int)x.l[i], src);
  return r;
}
BLS_INL fp2 fp2_shfl(const fp2& x, int src) { return fp2_make(fp_shfl(x.c0, src), fp_shfl(x.c1, src)); }
BLS_INL fp fp_keep(bool c, const fp& a) { return fp_select(c, a, fp_zero()); }
// lane groups of six (k_miller_acc6, gt6.hpp): ten per wave, lanes 60-63 idle
#define ACC6_GROUPS (WAVE / 6)
BLS_INL g2j g2j_xlane(const g2j& p) {
  g2j r;
  r.x = fp2_xlane(p.x);
  r.y = fp2_xlane(p.y);
  r.z = fp2_xlane(p.z);
  return r;
}
__device__ __forceinline__ g1a ld_pktab(const uint32_t* tab, uint32_t idx) {
  const uint4* q = reinterpret_cast<const uint4*>(tab + (size_t)idx * W_PKTAB);
  uint32_t w[W_PKTAB];
#pragma unroll
  for (int k = 0; k < W_PKTAB / 4; k++) {
    uint4 v = q[k];
    w[4 * k] = v.x;
    w[4 * k + 1] = v.y;
    w[4 * k + 2] = v.z;
    w[4 * k + 3] = v.w;
  }
  g1a r;
#pragma unroll
  for (int l = 0; l < BLS_NL; l++) {
    r.x.l[l] = w[l];
    r.y.l[l] = w[BLS_NL + l];
  }
  return r;
}

// [k]P for Jacobian P
template <class F>
__device__ jac<F> jac_mul_u64_j(const jac<F>& P, uint64_t k) {
  jac<F> r = jac_infinity<F>();
  if (k == 0) return r;
  int top = 63;
  while (((k >> top) & 1ull) == 0) top--;
  r = P;
  for (int i = top - 1; i >= 0; i--) {
    r = jac_dbl(r);
    if ((k >> i) & 1ull) r = jac_add(r, P);
  }
  return r;
}

// [r]P for the batch scalar encoded by the 64-bit word w (runtime.cpp `scalar words`):
//   r = a + b lambda (mod the group order),  lambda = -z^2 (curve.hpp endo_lambda: phi on G1, -psi^2 on G2),
//   a = sum_k d_k 16^k over the 8 nibbles of w's low half, b the same over its high half, d = 2 nibble - 15 (odd,
//   in [-15, 15]) -- so a = 2 lo + 1 - 2^32 and b = 2 hi + 1 - 2^32, odd 33-bit integers.
// The 2^64 words give 2^64 distinct r mod the group order (a collision would be a lattice vector (a - a', b - b') of
// x + y lambda = 0 with both coordinates below 2^33, but that lattice's shortest vectors, e.g. (z^2, 1), are ~2^127
// long), so the random linear combination keeps blst's 2^-64 soundness, while [r]P costs 28 doublings (8 windows of
// 4 bits, both halves sharing them: Straus) instead of the 60 of a 64-bit scalar.  Word 0 means r = 1 (CoreVerify),
// which the callers take as P itself.  Regular signed windows: every lane runs the same doublings and additions (no
// data-dependent branch); the table of odd multiples P, 3P, ..., 15P lives in HBM (SoA, tab[(e * 3 * WF + word) * n
// + i], WF = words of one coordinate) and lambda is applied to the entry the high half picks.
template <class F>
__device__ __forceinline__ void tab_st(uint32_t* tab, uint32_t n, uint32_t i, int e, const jac<F>& v) {
  constexpr int WF = sizeof(F) / 4;
  const uint32_t* s = reinterpret_cast<const uint32_t*>(&v);
#pragma unroll
  for (int w = 0; w < 3 * WF; w++) tab[((size_t)e * 3 * WF + w) * n + i] = s[w];
}
template <class F>
__device__ __forceinline__ jac<F> tab_ld(const uint32_t* tab, uint32_t n, uint32_t i, int e) {
  constexpr int WF = sizeof(F) / 4;
  jac<F> v;
  uint32_t* d = reinterpret_cast<uint32_t*>(&v);
#pragma unroll
  for (int w = 0; w < 3 * WF; w++) d[w] = tab[((size_t)e * 3 * WF + w) * n + i];
  return v;
}
// signed digit k (0..15) of word w: table entry (|d| - 1) / 2, sign
BLS_HD int scalar_word_digit(uint64_t w, int k, bool& neg) {
  const int d = 2 * (int)((w >> (4 * k)) & 15u) - 15;
  neg = d < 0;
  return (d < 0 ? -d : d) >> 1;
}
template <class F>
__device__ jac<F> jac_mul_scalar_word(const jac<F>& P, uint64_t w, uint32_t* tab, uint32_t n, uint32_t i) {
  const jac<F> P2 = jac_dbl(P);
  jac<F> t = P;
  tab_st(tab, n, i, 0, t);
#pragma unroll 1
  for (int e = 1; e < 8; e++) {
    t = jac_add(t, P2);
    tab_st(tab, n, i, e, t);
  }
  const uint32_t ii = opaque_u32(i);  // table addresses recomputed per window, not hoisted and spilled
  auto term = [&](int k, bool hi) {
    bool neg;
    const int e = scalar_word_digit(w, hi ? k + 8 : k, neg);
    jac<F> q = tab_ld<F>(tab, n, ii, e);
    if (hi) q = endo_lambda(q);
    return neg ? jac_neg(q) : q;
  };
  jac<F> r = jac_add(term(7, false), term(7, true));
#pragma unroll 1
  for (int k = 6; k >= 0; k--) {
    r = jac_dbl(jac_dbl(jac_dbl(jac_dbl(r))));
    r = jac_add(r, term(k, false));
    r = jac_add(r, term(k, true));
  }
  return r;
}

// [k]P for a multi-word scalar (little-endian 32-bit words), used by the workload-generation ops
template <class F>
__device__ jac<F> jac_mul_words(const jac<F>& P, const uint32_t* k, int nw) {
  jac<F> r = jac_infinity<F>();
  for (int i = 32 * nw - 1; i >= 0; i--) {
    r = jac_dbl(r);
    if ((k[i >> 5] >> (i & 31)) & 1u) r = jac_add(r, P);
  }
  return r;
}


// Small runs are latency-bound chains: a cooperative workgroup that shares its SIMDs with waves of the other branches'
// kernels issues at a fraction of its rate (k_miller_coop: 1.7 ms alone in tools/microbench/lat_probe.hip, 3-4 ms in
// a 128-set call's trace).  Launched with this much extra dynamic LDS, one such workgroup fills the CU's LDS (160 KB on
// gfx950) beyond what any other kernel of the pipeline needs (<= 36 KB), so the CU runs it alone.  0 when the device
// does not allow it (the launch then simply shares CUs).
// (One cached value per kernel and device: the template parameter is the kernel itself -- keyed by its type, kernels
// of one signature shared the first one's padding, and a larger kernel's static LDS plus that padding overflowed the
// CU -- and hipFuncSetAttribute applies to the current device only, so each device computes and sets its own.)
template <auto kernel>
inline size_t exclusive_cu_lds() {
  constexpr int kMaxDev = 64;
  static std::atomic<int64_t> cache[kMaxDev];  // zero-initialized: 0 = not yet computed, else pad + 1
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return 0;
  const int64_t c = cache[dev].load(std::memory_order_acquire);
  if (c) return (size_t)(c - 1);
  const size_t pad = [&]() -> size_t {
    int max_block = 0, per_cu = 0;
    if (hipDeviceGetAttribute(&max_block, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&per_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev) != hipSuccess)
      return 0;
    hipFuncAttributes a{};
    if (hipFuncGetAttributes(&a, reinterpret_cast<const void*>(kernel)) != hipSuccess) return 0;
    // leave less than the smallest other kernel's LDS (14 KB) free on the CU
    const size_t want = (size_t)per_cu - 8 * 1024;
    if (per_cu <= 0 || (size_t)max_block < want || a.sharedSizeBytes >= want) return 0;
    const size_t pad_b = want - a.sharedSizeBytes;
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)pad_b) != hipSuccess)
      return 0;
    return pad_b;
  }();
  cache[dev].store((int64_t)pad + 1, std::memory_order_release);
  return pad;
}

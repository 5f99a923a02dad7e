// Montgomery product forms for BLS12-381 Fp on gfx950 (verdict r4 #3: "microbenchmark the candidates first"):
//   mad64  14 x 28-bit limbs, v_mad_u64_u32 column sums (fp.hpp fp_mul_body, the product the stage kernels use)
//   u24    16 x 24-bit limbs, each limb product from v_mul_u32_u24 + v_mul_hi_u32_u24 into a 64-bit column sum
//   f64    16 x 24-bit limbs held in doubles, column sums by v_fma_f64 (exact below 2^53: 32 products of < 2^48),
//          carries and the Montgomery digit by floor / convert
//   mad64/24  16 x 24-bit limbs with v_mad_u64_u32 column sums (what the compiler makes of a 64-bit product of 24-bit
//          operands)
// Each lane runs a dependent chain x <- x * y (Montgomery) of ITERS products between a conversion into and out of its
// form's Montgomery domain, so every form computes the same integer x0 * y^ITERS mod p; the host compares the forms'
// results word for word and prints the first lanes' inputs and result for tools/microbench/limb_forms_check.py (Python
// big integers).  Rates at 1, 2 and 4 waves per SIMD (the kernels' register budget permitting).
// Status (profiles/r05_limb_forms.json): mad64 and f64 agree on every lane and with Python.  The 24-bit integer
// forms are not reliable on gfx950 with hipcc 7.2: u24 is wrong on every lane; mad64/24 was wrong on every lane until
// the g_dbg stores below were added, after which its chain is right and the extra x * y it stores is wrong (its x R
// and y R, second operand from constant memory, are right).  The same source built for the host (g++, clang -O3)
// is right on the same inputs.  Their rates stand as instruction-count evidence only.
//   python3 tools/microbench/gen_limb24.py
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/microbench/limb_forms.hip -o tools/microbench/limb_forms
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../lodestar_amd/csrc/fp.hpp"
#include "limb24_consts.h"

constexpr int ITERS = 1024;
constexpr int NSEED = 4096;

struct f24 {
  uint32_t l[16];
};
struct d24 {
  double l[16];
};

// ---------------------------------------------------------------------------------------------- u24
// FORM 1: the 48-bit limb product from v_mul_u32_u24 / v_mul_hi_u32_u24 (the high half through inline asm: written as a
// 64-bit product of 24-bit operands, the compiler folds multiply and column add into v_mad_u64_u32 -- FORM 3)
template <bool U24>
__device__ __forceinline__ uint64_t mul24(uint32_t a, uint32_t b) {
  if constexpr (U24) {
    uint32_t hi;
    asm("v_mul_hi_u32_u24 %0, %1, %2" : "=v"(hi) : "v"(a), "v"(b));
    return ((uint64_t)hi << 32) | __umul24(a, b);
  } else {
    return (uint64_t)a * b;  // limbs < 2^24 by construction: v_mad_u64_u32 with no 24-bit product instruction
  }
}
// a, b < 2p (limbs < 2^24), result < 2p (4p < 2^384)
template <bool U24>
__device__ __forceinline__ f24 u24_mul(const f24& a, const f24& b) {
  f24 r;
  uint32_t m[16];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 16; k++) {
#pragma unroll
    for (int i = 0; i <= k; i++) acc += mul24<U24>(a.l[i], b.l[k - i]);
#pragma unroll
    for (int i = 0; i < k; i++) acc += mul24<U24>(m[i], L24_P[k - i]);
    // the digit's 24-bit mask through asm (a plain `& 0xFFFFFF` after __umul24 was dropped by hipcc 7.2 here)
    uint32_t mk = (uint32_t)acc * L24_N0;  // low 24 bits depend only on acc's low 24 bits
    asm("v_and_b32 %0, 0xffffff, %1" : "=v"(mk) : "v"(mk));
    m[k] = mk;
    acc += mul24<U24>(mk, L24_P[0]);
    acc >>= 24;
  }
#pragma unroll
  for (int k = 16; k < 31; k++) {
#pragma unroll
    for (int i = k - 15; i < 16; i++) {
      acc += mul24<U24>(a.l[i], b.l[k - i]);
      acc += mul24<U24>(m[i], L24_P[k - i]);
    }
    r.l[k - 16] = (uint32_t)acc & 0xFFFFFFu;
    acc >>= 24;
  }
  r.l[15] = (uint32_t)acc;
  return r;
}

// ---------------------------------------------------------------------------------------------- f64
__device__ __forceinline__ double d_floor24(double x) { return __builtin_floor(x * 0x1p-24); }
__device__ __forceinline__ d24 f64_mul(const d24& a, const d24& b) {
  d24 r;
  double m[16];
  double acc = 0.0;
#pragma unroll
  for (int k = 0; k < 16; k++) {
#pragma unroll
    for (int i = 0; i <= k; i++) acc = __builtin_fma(a.l[i], b.l[k - i], acc);
#pragma unroll
    for (int i = 0; i < k; i++) acc = __builtin_fma(m[i], (double)L24_P[k - i], acc);
    const double q = d_floor24(acc);
    const uint32_t lo = (uint32_t)__builtin_fma(-q, 0x1p24, acc);  // acc mod 2^24, exact
    const double mk = (double)(__umul24(lo, L24_N0) & 0xFFFFFFu);
    m[k] = mk;
    acc = __builtin_fma(mk, (double)L24_P[0], acc);  // now a multiple of 2^24
    acc = acc * 0x1p-24;
  }
#pragma unroll
  for (int k = 16; k < 31; k++) {
#pragma unroll
    for (int i = k - 15; i < 16; i++) {
      acc = __builtin_fma(a.l[i], b.l[k - i], acc);
      acc = __builtin_fma(m[i], (double)L24_P[k - i], acc);
    }
    const double q = d_floor24(acc);
    r.l[k - 16] = __builtin_fma(-q, 0x1p24, acc);
    acc = q;
  }
  r.l[15] = acc;
  return r;
}

// ---------------------------------------------------------------------------------------------- kernels
// in: per seed, x0 and y as 16 x 24-bit limbs (plain integers < p) and as 14 x 28-bit limbs.  out: per lane, the
// canonical result as 16 x 24-bit limbs.
__device__ __forceinline__ void canon24(uint32_t* w) {  // w < 2p -> w mod p (24-bit limbs)
  uint32_t t[16];
  int32_t bw = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const int32_t v = (int32_t)w[i] - (int32_t)L24_P[i] + bw;
    t[i] = (uint32_t)v & 0xFFFFFFu;
    bw = v >> 24;
  }
  if (bw == 0)
#pragma unroll
    for (int i = 0; i < 16; i++) w[i] = t[i];
}

__device__ uint32_t g_dbg[4][16];  // lane 0 of the 24-bit integer form: x R, y R, x R y, x after the chain
template <int FORM>
__global__ __launch_bounds__(64) void k_chain(const uint32_t* in24, const uint32_t* in28, uint32_t* out) {
  const uint32_t lane = blockIdx.x * 64 + threadIdx.x;
  const uint32_t s = lane % NSEED;
  uint32_t res[16];
  if constexpr (FORM == 0) {
    fp x, y;
#pragma unroll
    for (int i = 0; i < BLS_NL; i++) {
      x.l[i] = in28[(2 * s) * BLS_NL + i];
      y.l[i] = in28[(2 * s + 1) * BLS_NL + i];
    }
    x = fp_mul_body(x, FP_R2);
    y = fp_mul_body(y, FP_R2);
#pragma unroll 1
    for (int it = 0; it < ITERS; it++) x = fp_mul_body(x, y);
    fp one = fp_zero();
    one.l[0] = 1;
    x = fp_canon(fp_mul_body(x, one));
    // 28-bit limbs -> 24-bit limbs
    int bit = 0;
#pragma unroll
    for (int j = 0; j < 16; j++) res[j] = 0;
    for (int i = 0; i < BLS_NL; i++)
      for (int b = 0; b < 28; b++, bit++)
        if (bit < 384) res[bit / 24] |= ((x.l[i] >> b) & 1u) << (bit % 24);
  } else if constexpr (FORM == 1 || FORM == 3) {
    constexpr bool U24 = FORM == 1;
    f24 x, y, r2, one;
#pragma unroll
    for (int i = 0; i < 16; i++) {
      x.l[i] = in24[(2 * s) * 16 + i];
      y.l[i] = in24[(2 * s + 1) * 16 + i];
      r2.l[i] = L24_R2[i];
      one.l[i] = i == 0;
    }
    x = u24_mul<U24>(x, r2);
    y = u24_mul<U24>(y, r2);
    const f24 xy = u24_mul<U24>(x, y);
    if (FORM == 3 && lane == 0)
      for (int i = 0; i < 16; i++) {
        g_dbg[0][i] = x.l[i];
        g_dbg[1][i] = y.l[i];
        g_dbg[2][i] = xy.l[i];
      }
#pragma unroll 1
    for (int it = 0; it < ITERS; it++) x = u24_mul<U24>(x, y);
    if (FORM == 3 && lane == 0)
      for (int i = 0; i < 16; i++) g_dbg[3][i] = x.l[i];
    x = u24_mul<U24>(x, one);
#pragma unroll
    for (int i = 0; i < 16; i++) res[i] = x.l[i];
    canon24(res);
  } else {
    d24 x, y, r2, one;
#pragma unroll
    for (int i = 0; i < 16; i++) {
      x.l[i] = (double)in24[(2 * s) * 16 + i];
      y.l[i] = (double)in24[(2 * s + 1) * 16 + i];
      r2.l[i] = (double)L24_R2[i];
      one.l[i] = i == 0 ? 1.0 : 0.0;
    }
    x = f64_mul(x, r2);
    y = f64_mul(y, r2);
#pragma unroll 1
    for (int it = 0; it < ITERS; it++) x = f64_mul(x, y);
    x = f64_mul(x, one);
#pragma unroll
    for (int i = 0; i < 16; i++) res[i] = (uint32_t)x.l[i];
    canon24(res);
  }
#pragma unroll
  for (int i = 0; i < 16; i++) out[(size_t)lane * 16 + i] = res[i];
}

#define CHK(x)                                                \
  do {                                                        \
    hipError_t e_ = (x);                                      \
    if (e_ != hipSuccess) {                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); \
      exit(1);                                                \
    }                                                         \
  } while (0)

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint32_t next32() {
  rng ^= rng << 13;
  rng ^= rng >> 7;
  rng ^= rng << 17;
  return (uint32_t)(rng >> 11);
}

template <class K>
static double run(K kern, int waves, const uint32_t* d24in, const uint32_t* d28in, uint32_t* d_out) {
  hipLaunchKernelGGL(kern, dim3(waves), dim3(64), 0, 0, d24in, d28in, d_out);  // warm
  CHK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  CHK(hipEventRecord(a, 0));
  hipLaunchKernelGGL(kern, dim3(waves), dim3(64), 0, 0, d24in, d28in, d_out);
  CHK(hipEventRecord(b, 0));
  CHK(hipEventSynchronize(b));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, a, b));
  return ms;
}

int main() {
  // inputs: random 380-bit integers (< p: bit 380 and above clear; p > 2^380)
  static uint32_t bits[2 * NSEED][12];
  static uint32_t h24[2 * NSEED * 16], h28[2 * NSEED * BLS_NL];
  for (int v = 0; v < 2 * NSEED; v++) {
    for (int w = 0; w < 12; w++) bits[v][w] = next32();
    bits[v][11] &= 0x0FFFFFFFu;  // < 2^380
    for (int j = 0; j < 16; j++) h24[v * 16 + j] = 0;
    for (int j = 0; j < BLS_NL; j++) h28[v * BLS_NL + j] = 0;
    for (int b = 0; b < 384; b++) {
      const uint32_t bit = (bits[v][b / 32] >> (b % 32)) & 1u;
      h24[v * 16 + b / 24] |= bit << (b % 24);
      h28[v * BLS_NL + b / 28] |= bit << (b % 28);
    }
  }
  const int max_waves = 1024 * 4;
  uint32_t *d24in, *d28in, *dout[4];
  CHK(hipMalloc(&d24in, sizeof(h24)));
  CHK(hipMalloc(&d28in, sizeof(h28)));
  CHK(hipMemcpy(d24in, h24, sizeof(h24), hipMemcpyHostToDevice));
  CHK(hipMemcpy(d28in, h28, sizeof(h28), hipMemcpyHostToDevice));
  const size_t out_words = (size_t)max_waves * 64 * 16;
  for (int f = 0; f < 4; f++) CHK(hipMalloc(&dout[f], out_words * 4));
  const char* names[4] = {"mad64 (14 x 28-bit, fp_mul_body)", "u24 (16 x 24-bit, mul_u24 / mul_hi_u24 + 64-bit add)",
                          "f64 (16 x 24-bit, fma_f64)", "mad64 over 16 x 24-bit limbs"};
  printf("{\"tool\": \"tools/microbench/limb_forms.hip\", \"iters\": %d, \"results\": [\n", ITERS);
  bool first = true;
  for (int wps : {1, 2, 4}) {
    const int waves = 1024 * wps;
    double ms[4];
    ms[0] = run(k_chain<0>, waves, d24in, d28in, dout[0]);
    ms[1] = run(k_chain<1>, waves, d24in, d28in, dout[1]);
    ms[2] = run(k_chain<2>, waves, d24in, d28in, dout[2]);
    ms[3] = run(k_chain<3>, waves, d24in, d28in, dout[3]);
    for (int f = 0; f < 4; f++) {
      const double rate = (double)waves * 64 * ITERS / (ms[f] * 1e-3);
      printf("%s  {\"form\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"mont_products_per_s\": %.4e}", first ? "" : ",\n",
             names[f], wps, ms[f], rate);
      first = false;
    }
  }
  // cross-check the forms' results (last launch: 4 waves per SIMD, every lane)
  static uint32_t o[4][(size_t)1024 * 4 * 64 * 16];
  for (int f = 0; f < 4; f++) CHK(hipMemcpy(o[f], dout[f], out_words * 4, hipMemcpyDeviceToHost));
  size_t bad1 = 0, bad2 = 0, bad3 = 0;
  for (size_t i = 0; i < out_words; i += 16) {
    if (memcmp(o[0] + i, o[1] + i, 64)) bad1++;
    if (memcmp(o[0] + i, o[2] + i, 64)) bad2++;
    if (memcmp(o[0] + i, o[3] + i, 64)) bad3++;
  }
  printf("\n], \"lanes_checked\": %zu, \"u24_mismatches\": %zu, \"f64_mismatches\": %zu, \"mad64_24_mismatches\": %zu, \"samples\": [\n",
         out_words / 16, bad1, bad2, bad3);
  for (int s = 0; s < 4; s++) {
    auto hex = [](const uint32_t* l24) {
      static char buf[6][128];
      static int k = 0;
      char* b = buf[k++ % 6];
      char* p = b;
      for (int j = 15; j >= 0; j--) p += sprintf(p, "%06x", l24[j]);
      return (const char*)b;
    };
    printf("  {\"x0\": \"%s\", \"y\": \"%s\", \"x\": \"%s\",", hex(h24 + (2 * s) * 16), hex(h24 + (2 * s + 1) * 16),
           hex(o[0] + (size_t)s * 16));
    printf(" \"x_u24\": \"%s\", \"x_f64\": \"%s\", \"x_mad64_24\": \"%s\"}%s\n", hex(o[1] + (size_t)s * 16),
           hex(o[2] + (size_t)s * 16), hex(o[3] + (size_t)s * 16), s < 3 ? "," : "");
  }
  uint32_t dbg[4][16];
  CHK(hipMemcpyFromSymbol(dbg, HIP_SYMBOL(g_dbg), sizeof(dbg)));
  printf("], \"debug_lane0_form3\": [");
  for (int j = 0; j < 4; j++) {
    printf("\"");
    for (int i = 15; i >= 0; i--) printf("%08x", dbg[j][i]);
    printf("\"%s", j < 3 ? ", " : "");
  }
  printf("]}\n");
  return 0;
}

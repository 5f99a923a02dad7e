// Latency probe of the serial building blocks (one workgroup, timestamps from the GPU's constant-rate wall clock):
// single-lane chains (Montgomery product, Fp2 product, the two inversions, the (p-3)/4 exponentiation, a G2
// Jacobian doubling) and the 128-lane cooperative Fp12 steps of gt_wave.hpp (cyclotomic squaring, dense and sparse
// products, the whole final exponentiation).  Prints one JSON object: microseconds per operation.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include tools/microbench/lat_probe.hip -o tools/microbench/lat_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../../lodestar_amd/csrc/gt_wave.hpp"
#include "../../lodestar_amd/csrc/g2_coop.hpp"

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

enum { P_MUL, P_SQR, P_FP2MUL, P_INV, P_INVPOW, P_POW34, P_G2DBL, P_CYC, P_GMUL, P_GSPARSE, P_FINEXP, P_FP12INV, P_CYC1,
       P_CYC2, P_SYNC, P_LACC, P_G2C, P_G2C_P1, P_G2C_R1, P_G2ADD, P_G2ADDAFF, P_MILLER, P_FP12MUL, P_G2CADD, NP };
static const char* NAMES[NP] = {"fp_mul", "fp_sqr", "fp2_mul", "fp_inv_divsteps", "fp_inv_pow", "fp_pow_p34",
                                "g2_jac_dbl", "gtw_cyc_sqr", "gtw_mul", "gtw_mul_sparse", "gtw_final_exp",
                                "fp12_inv_lane0", "gtw_cyc_sqr_products", "gtw_cyc_sqr_recombine", "gtw_sync",
                                "lacc_fin_lane", "g2c_dbl", "g2c_dbl_p1", "g2c_dbl_r1", "g2_jac_add", "g2_jac_add_aff",
                                "gtw_miller_loop", "fp12_mul_lane", "g2c_add"};
static const int REPS[NP] = {256, 256, 128, 8, 4, 4, 32, 64, 32, 32, 1, 2, 64, 64, 256, 256, 64, 64, 64, 16, 16, 1, 16, 32};

__device__ __forceinline__ uint64_t now() { return wall_clock64(); }

__global__ __launch_bounds__(GTW_MILLER_LANES) void k_probe(uint64_t* ticks, uint32_t seed, uint32_t* sink) {
  __shared__ GtwLds sh;
  __shared__ uint32_t g2lds[(GTW_MILLER_LANES / G2C_LANES) * G2C_WORDS];
  const uint32_t t = threadIdx.x;
  fp a, b;
  for (int i = 0; i < BLS_NL; i++) {
    a.l[i] = (seed * 2654435761u + i * 40503u + t) & BLS_MASK;
    b.l[i] = (seed * 97u + i * 7919u + 3 * t) & BLS_MASK;
  }
  a.l[BLS_NL - 1] &= 0xffff;
  b.l[BLS_NL - 1] &= 0xffff;
  // Fp12 values in LDS
  for (uint32_t w = t; w < (GTW_MILLER_LANES / G2C_LANES) * G2C_WORDS; w += GTW_MILLER_LANES) g2lds[w] = (seed * 7 + 11 * w) & 0xFFFFFFu;
  for (uint32_t w = t; w < 12 * BLS_NL; w += GTW_LANES) {
    sh.F[w] = (seed + 31 * w) & BLS_MASK;
    sh.G[w] = (seed * 3 + 17 * w) & BLS_MASK;
    sh.L[w] = (seed * 5 + 13 * w) & BLS_MASK;
  }
  gtw_sync();
  uint32_t acc = 0;
  for (int p = 0; p < NP; p++) {
    gtw_sync();
    const uint64_t t0 = now();
    for (int r = 0; r < REPS[p]; r++) {
      switch (p) {
        case P_MUL: if (t == 0) a = fp_mul(a, b); break;
        case P_SQR: if (t == 0) a = fp_sqr(a); break;
        case P_FP2MUL: if (t == 0) { fp2 x = fp2_make(a, b), y = fp2_make(b, a); x = fp2_mul(x, y); a = x.c0; b = x.c1; } break;
        case P_INV: if (t == 0) a = fp_inv(a); break;
        case P_INVPOW: if (t == 0) a = fp_inv_pow(a); break;
        case P_POW34: if (t == 0) a = fp_pow_p34(a); break;
        case P_G2DBL: if (t == 0) { g2j q; q.x = fp2_make(a, b); q.y = fp2_make(b, a); q.z = fp2_make(a, a); q = jac_dbl(q); a = q.x.c0; b = q.y.c1; } break;
        case P_CYC: gtw_cyc_sqr(sh.F, sh.F, sh.S, t); break;
        case P_GMUL: gtw_mul<false>(sh.F, sh.F, sh.G, sh.S, t); break;
        case P_GSPARSE: gtw_mul<true>(sh.F, sh.F, sh.L, sh.S, t); break;
        case P_FINEXP: gtw_final_exp(sh.F, sh.W, sh.S, t); break;
        case P_FP12INV: if (t == 0) gtw_from_reg(sh.G, fp12_inv(gtw_to_reg(sh.F))); break;
        case P_CYC1: gtw_cyc_sqr<1>(sh.F, sh.F, sh.S, t); break;
        case P_CYC2: gtw_cyc_sqr<2>(sh.F, sh.F, sh.S, t); break;
        case P_SYNC: gtw_sync(); break;
        case P_G2C: g2c_dbl(g2lds + (t / G2C_LANES) * G2C_WORDS, t % G2C_LANES); break;
        case P_G2CADD: g2c_add(g2lds + (t / G2C_LANES) * G2C_WORDS, t % G2C_LANES); break;
        case P_G2C_P1: g2c_dbl_p1(g2lds + (t / G2C_LANES) * G2C_WORDS, t % G2C_LANES); gtw_sync(); break;
        case P_G2C_R1: g2c_dbl_r1(g2lds + (t / G2C_LANES) * G2C_WORDS, t % G2C_LANES); gtw_sync(); break;
        case P_G2ADD: if (t == 0) { g2j q, r; q.x = fp2_make(a, b); q.y = fp2_make(b, a); q.z = fp2_make(a, a); r.x = fp2_make(b, b); r.y = fp2_make(a, b); r.z = fp2_make(b, a); q = jac_add(q, r); a = q.x.c0; b = q.y.c1; } break;
        case P_G2ADDAFF: if (t == 0) { g2j q; g2a r; q.x = fp2_make(a, b); q.y = fp2_make(b, a); q.z = fp2_make(a, a); r.x = fp2_make(b, b); r.y = fp2_make(a, b); q = jac_add_aff(q, r); a = q.x.c0; b = q.y.c1; } break;
        case P_MILLER: { if (t < 4) lds_st(sh.QA, t, t & 1 ? a : b); gtw_sync(); gtw_miller_loop(sh.G, sh.QA, a, b, sh.TB, sh.L, sh.L1, sh.S, sh.S2, t); } break;
        case P_FP12MUL: if (t == 0) { fp12 x = gtw_to_reg(sh.F), y = gtw_to_reg(sh.G); gtw_from_reg(sh.G, fp12_mul(x, y)); } break;
        case P_LACC: if (t == 0) { lacc q; for (int i = 0; i < BLS_NL; i++) { q.pos[i] = a.l[i]; q.neg[i] = b.l[i]; } a = lacc_fin(q); } break;
      }
    }
    gtw_sync();
    const uint64_t t1 = now();
    if (t == 0) ticks[p] = t1 - t0;
  }
  for (int i = 0; i < BLS_NL; i++) acc ^= a.l[i] ^ b.l[i] ^ sh.F[i] ^ sh.G[i];
  if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
  uint64_t* d;
  uint32_t* sink;
  CHECK(hipMalloc(&d, NP * 8));
  CHECK(hipMalloc(&sink, 4));
  int rate_khz = 0;
  CHECK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0));
  hipLaunchKernelGGL(k_probe, dim3(1), dim3(GTW_MILLER_LANES), 0, 0, d, 1u, sink);  // warm-up (code fetch)
  CHECK(hipDeviceSynchronize());
  hipLaunchKernelGGL(k_probe, dim3(1), dim3(GTW_MILLER_LANES), 0, 0, d, 2u, sink);
  CHECK(hipDeviceSynchronize());
  uint64_t h[NP];
  CHECK(hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost));
  printf("{\"wall_clock_khz\": %d, \"us_per_op\": {", rate_khz);
  for (int p = 0; p < NP; p++)
    printf("%s\"%s\": %.3f", p ? ", " : "", NAMES[p], 1e3 * (double)h[p] / rate_khz / REPS[p]);
  printf("}}\n");
  return 0;
}

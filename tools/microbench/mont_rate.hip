// Montgomery-product throughput vs waves per SIMD on gfx950: how much of the VALU a lane-per-element
// design gets at 1, 2, 4 and 8 resident waves per SIMD.  Each lane runs a dependent chain of products
// (the shape of the stage kernels: one long serial computation per lane), with the product either as the
// register-ABI call of fp.hpp (fp_mul) or as the Fp2 Karatsuba product (3 products + 5 add/sub).
//   hipcc -O3 --offload-arch=gfx950 -I include tools/microbench/mont_rate.hip -o tools/microbench/mont_rate
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../../lodestar_amd/csrc/tower.hpp"
#include "fp_mad.hpp"

#if defined(__HIP_DEVICE_COMPILE__)
__device__ __noinline__ fp_ret fp_mul_r_mad(BLS_PARAMS14(a), BLS_PARAMS14(b)) {
  const fp x = BLS_INIT14(a), y = BLS_INIT14(b);
  const fp r = fp_mul_body_mad(x, y);
  fp_ret o;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) o.l[i] = r.l[i];
  return o;
}
__device__ __noinline__ fp_ret fp_sqr_r_mad(BLS_PARAMS14(a)) {
  const fp x = BLS_INIT14(a);
  const fp r = fp_sqr_body_mad(x);
  fp_ret o;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) o.l[i] = r.l[i];
  return o;
}
__device__ __forceinline__ fp fp_mul_mad(const fp& a, const fp& b) {
  const fp_ret t = fp_mul_r_mad(BLS_ARGS14(a), BLS_ARGS14(b));
  fp r;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) r.l[i] = t.l[i];
  return r;
}
__device__ __forceinline__ fp fp_sqr_mad(const fp& a) {
  const fp_ret t = fp_sqr_r_mad(BLS_ARGS14(a));
  fp r;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) r.l[i] = t.l[i];
  return r;
}
#endif

// correctness: the explicit-MAD bodies against fp.hpp's on pseudo-random operands (limbs < 2^30 / 2^29)
__global__ __launch_bounds__(64) void k_check(uint32_t* bad, uint32_t s) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t x = threadIdx.x * 2654435761u + blockIdx.x * 40503u + s;
  auto rnd = [&]() { x ^= x << 13; x ^= x >> 17; x ^= x << 5; return x; };
  for (int it = 0; it < 64; it++) {
    fp a, b, c;
    for (int i = 0; i < BLS_NL; i++) {
      a.l[i] = rnd() & 0x3FFFFFFFu;
      b.l[i] = rnd() & 0x3FFFFFFFu;
      c.l[i] = rnd() & 0x1FFFFFFFu;
    }
    a.l[BLS_NL - 1] &= 0x3FFFFu;
    b.l[BLS_NL - 1] &= 0x3FFFFu;
    c.l[BLS_NL - 1] &= 0x3FFFFu;
    const fp r0 = fp_mul(a, b), r1 = fp_mul_mad(a, b), q0 = fp_sqr(c), q1 = fp_sqr_mad(c);
    for (int i = 0; i < BLS_NL; i++)
      if (r0.l[i] != r1.l[i] || q0.l[i] != q1.l[i]) atomicAdd(bad, 1u);
  }
#endif
}

__global__ __launch_bounds__(64) void k_fp_mul_mad(uint32_t* out, uint32_t s) {
#if defined(__HIP_DEVICE_COMPILE__)
  fp a, b;
  for (int i = 0; i < BLS_NL; i++) {
    a.l[i] = (threadIdx.x * 7919u + i * 104729u + s) & BLS_MASK;
    b.l[i] = (threadIdx.x * 31u + i * 7u + s) & BLS_MASK;
  }
  a.l[BLS_NL - 1] &= 0xFFFFu;
  b.l[BLS_NL - 1] &= 0xFFFFu;
#pragma unroll 1
  for (int it = 0; it < 256; it++) {
    a = fp_mul_mad(a, b);
    b = fp_mul_mad(b, a);
  }
  uint32_t r = 0;
  for (int i = 0; i < BLS_NL; i++) r ^= a.l[i] ^ b.l[i];
  if (r == 0x1234567u) out[0] = r;
#endif
}

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int ITERS = 256;

__global__ __launch_bounds__(64) void k_fp_mul(uint32_t* out, uint32_t s) {
  fp a, b;
  for (int i = 0; i < BLS_NL; i++) {
    a.l[i] = (threadIdx.x * 7919u + i * 104729u + s) & BLS_MASK;
    b.l[i] = (threadIdx.x * 31u + i * 7u + s) & BLS_MASK;
  }
  a.l[BLS_NL - 1] &= 0xFFFFu;
  b.l[BLS_NL - 1] &= 0xFFFFu;
#pragma unroll 1
  for (int it = 0; it < ITERS; it++) {
    a = fp_mul(a, b);
    b = fp_mul(b, a);
  }
  uint32_t r = 0;
  for (int i = 0; i < BLS_NL; i++) r ^= a.l[i] ^ b.l[i];
  if (r == 0x1234567u) out[0] = r;
}

__global__ __launch_bounds__(64) void k_fp2_mul(uint32_t* out, uint32_t s) {
  fp2 a, b;
  for (int i = 0; i < BLS_NL; i++) {
    a.c0.l[i] = (threadIdx.x * 7919u + i * 104729u + s) & BLS_MASK;
    a.c1.l[i] = (threadIdx.x * 17u + i * 1049u + s) & BLS_MASK;
    b.c0.l[i] = (threadIdx.x * 31u + i * 7u + s) & BLS_MASK;
    b.c1.l[i] = (threadIdx.x * 3u + i * 77u + s) & BLS_MASK;
  }
  a.c0.l[BLS_NL - 1] &= 0xFFFFu;
  a.c1.l[BLS_NL - 1] &= 0xFFFFu;
  b.c0.l[BLS_NL - 1] &= 0xFFFFu;
  b.c1.l[BLS_NL - 1] &= 0xFFFFu;
#pragma unroll 1
  for (int it = 0; it < ITERS / 2; it++) {
    a = fp2_mul(a, b);
    b = fp2_mul(b, a);
  }
  uint32_t r = 0;
  for (int i = 0; i < BLS_NL; i++) r ^= a.c0.l[i] ^ b.c1.l[i];
  if (r == 0x1234567u) out[0] = r;
}

typedef void (*kfn)(uint32_t*, uint32_t);

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int simds = prop.multiProcessorCount * 4;
  uint32_t* d;
  CHECK(hipMalloc(&d, 64));
  struct { const char* name; kfn f; double products_per_lane; } ks[] = {
      {"fp_mul (register-ABI call)", k_fp_mul, 2.0 * ITERS},
      {"fp2_mul (3 products + add/sub)", k_fp2_mul, 3.0 * ITERS},
      {"fp_mul explicit MADs (2 chains, rotated carry SGPRs)", k_fp_mul_mad, 2.0 * ITERS},
  };
  {
    uint32_t* bad;
    CHECK(hipMalloc(&bad, 4));
    CHECK(hipMemset(bad, 0, 4));
    hipLaunchKernelGGL(k_check, dim3(1024), dim3(64), 0, 0, bad, 7u);
    CHECK(hipDeviceSynchronize());
    uint32_t h = 0;
    CHECK(hipMemcpy(&h, bad, 4, hipMemcpyDeviceToHost));
    printf("{\"check_mismatched_limbs\": %u, \"cases\": %d},\n", h, 1024 * 64 * 64 * 2);
  }
  printf("{\"device\": \"%s\", \"simds\": %d, \"results\": [\n", prop.gcnArchName, simds);
  bool first = true;
  for (auto& k : ks) {
    for (int wps : {1, 2, 3, 4, 8}) {
      const int grid = simds * wps;  // one 64-lane wave per block
      hipLaunchKernelGGL(k.f, dim3(grid), dim3(64), 0, 0, d, 1u);
      CHECK(hipDeviceSynchronize());
      hipEvent_t e0, e1;
      CHECK(hipEventCreate(&e0));
      CHECK(hipEventCreate(&e1));
      CHECK(hipEventRecord(e0));
      const int reps = 3;
      for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k.f, dim3(grid), dim3(64), 0, 0, d, (uint32_t)r);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      const double prods = k.products_per_lane * grid * 64.0 * reps;
      printf("%s  {\"kernel\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"mont_products_per_s\": %.4e, "
             "\"v_mad_per_s\": %.4e}",
             first ? "" : ",\n", k.name, wps, ms / reps, prods / (ms * 1e-3), prods * 392 / (ms * 1e-3));
      first = false;
    }
  }
  printf("\n]}\n");
  return 0;
}

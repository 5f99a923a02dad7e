// Fp2 multiplication throughput at 1 and 2 resident waves per SIMD, each lane a dependent chain of fp2_mul
// (the shape of the stage kernels).  Variants:
//   call3       tower.hpp fp2_mul: three register-ABI product calls (fp_mul_r) + 3 subtractions (the pipeline today)
//   lazy_inl    fp2_mul_lazy_body inlined: lazy reduction (5 x 196 MADs), five interleaved MAD chains
//   lazy_lds    the same body behind ONE noinline call: a0, a1 as the 28 register arguments, b0, b1 through a
//               per-lane LDS slot (the AMDGPU calling convention passes only 32 VGPR arguments in registers)
// plus a correctness pass comparing lazy_lds with call3 (canonical values) on pseudo-random operands.
//   hipcc -O3 --offload-arch=gfx950 -I include tools/microbench/fp2_rate.hip -o tools/microbench/fp2_rate
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../../lodestar_amd/csrc/tower.hpp"

constexpr int ITERS = 128;
constexpr int LDS_LANES = 64;

#if defined(__HIP_DEVICE_COMPILE__)
__shared__ uint32_t g_fp2_b[2 * BLS_NL * LDS_LANES];
struct fp_ret2 {
  uint32_t l[2 * BLS_NL];
};
__device__ __noinline__ fp_ret2 fp2_mul_lds_r(BLS_PARAMS14(a), BLS_PARAMS14(c)) {
  const fp x0 = BLS_INIT14(a), x1 = BLS_INIT14(c);
  const uint32_t t = threadIdx.x;
  fp y0, y1;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) {
    y0.l[i] = g_fp2_b[i * LDS_LANES + t];
    y1.l[i] = g_fp2_b[(BLS_NL + i) * LDS_LANES + t];
  }
  const fp2 r = fp2_mul_lazy_body(x0, x1, y0, y1);
  fp_ret2 o;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) {
    o.l[i] = r.c0.l[i];
    o.l[BLS_NL + i] = r.c1.l[i];
  }
  return o;
}
__device__ __forceinline__ fp2 fp2_mul_lds(const fp2& a, const fp2& b) {
  const uint32_t t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) {
    g_fp2_b[i * LDS_LANES + t] = b.c0.l[i];
    g_fp2_b[(BLS_NL + i) * LDS_LANES + t] = b.c1.l[i];
  }
  const fp_ret2 o = fp2_mul_lds_r(BLS_ARGS14(a.c0), BLS_ARGS14(a.c1));
  fp2 r;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) {
    r.c0.l[i] = o.l[i];
    r.c1.l[i] = o.l[BLS_NL + i];
  }
  return r;
}
#endif

__device__ __forceinline__ void seed2(fp2& a, uint32_t t, uint32_t k, uint32_t s) {
  for (int i = 0; i < BLS_NL; i++) {
    a.c0.l[i] = (t * (7919u + 2 * k) + i * (104729u + k) + s) & BLS_MASK;
    a.c1.l[i] = (t * (17u + 4 * k) + i * (1049u + 3 * k) + s) & BLS_MASK;
  }
  a.c0.l[BLS_NL - 1] &= 0xFFFFu;
  a.c1.l[BLS_NL - 1] &= 0xFFFFu;
}
__device__ __forceinline__ void sink2(uint32_t* out, const fp2& a) {
  uint32_t r = 0;
  for (int i = 0; i < BLS_NL; i++) r ^= a.c0.l[i] ^ a.c1.l[i];
  if (r == 0x1234567u) out[0] = r;
}

template <int V>
__global__ __launch_bounds__(64) void k_rate(uint32_t* out, uint32_t s) {
#if defined(__HIP_DEVICE_COMPILE__)
  fp2 a, b;
  seed2(a, threadIdx.x, 0, s);
  seed2(b, threadIdx.x, 1, s);
#pragma unroll 1
  for (int it = 0; it < ITERS; it++) {
    if constexpr (V == 0) {
      a = fp2_mul(a, b);
      b = fp2_mul(b, a);
    } else if constexpr (V == 1) {
      a = fp2_mul_lazy_body(a.c0, a.c1, b.c0, b.c1);
      b = fp2_mul_lazy_body(b.c0, b.c1, a.c0, a.c1);
    } else {
      a = fp2_mul_lds(a, b);
      b = fp2_mul_lds(b, a);
    }
  }
  sink2(out, a);
  sink2(out, b);
#endif
}

__global__ __launch_bounds__(64) void k_check(uint32_t* bad, uint32_t s) {
#if defined(__HIP_DEVICE_COMPILE__)
  fp2 a, b;
  seed2(a, threadIdx.x + 64 * blockIdx.x, 5, s);
  seed2(b, threadIdx.x + 64 * blockIdx.x, 9, s);
  for (int it = 0; it < 16; it++) {
    const fp2 r0 = fp2_mul(a, b), r1 = fp2_mul_lds(a, b);
    const fp c00 = fp_canon(r0.c0), c01 = fp_canon(r0.c1), c10 = fp_canon(r1.c0), c11 = fp_canon(r1.c1);
    for (int i = 0; i < BLS_NL; i++)
      if (c00.l[i] != c10.l[i] || c01.l[i] != c11.l[i]) atomicAdd(bad, 1u);
    a = r0;
    b = fp2_add(r1, b);
  }
#endif
}

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
typedef void (*kfn)(uint32_t*, uint32_t);

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int simds = prop.multiProcessorCount * 4;
  uint32_t *d, *bad;
  CHECK(hipMalloc(&d, 64));
  CHECK(hipMalloc(&bad, 4));
  CHECK(hipMemset(bad, 0, 4));
  hipLaunchKernelGGL(k_check, dim3(1024), dim3(64), 0, 0, bad, 3u);
  CHECK(hipDeviceSynchronize());
  uint32_t h = 0;
  CHECK(hipMemcpy(&h, bad, 4, hipMemcpyDeviceToHost));
  printf("{\"device\": \"%s\", \"simds\": %d, \"check_mismatched_limbs\": %u, \"check_cases\": %d, \"results\": [\n",
         prop.gcnArchName, simds, h, 1024 * 64 * 16);
  struct { const char* name; kfn f; } ks[] = {{"call3", k_rate<0>}, {"lazy_inl", k_rate<1>}, {"lazy_lds", k_rate<2>}};
  bool first = true;
  for (auto& k : ks) {
    for (int wps : {1, 2}) {
      const int grid = simds * wps;
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
      const double n = 2.0 * ITERS * grid * 64.0 * reps;
      printf("%s  {\"kernel\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"fp2_mul_per_s\": %.4e}", first ? "" : ",\n",
             k.name, wps, ms / reps, n / (ms * 1e-3));
      first = false;
    }
  }
  printf("\n]}\n");
  return 0;
}

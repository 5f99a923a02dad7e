// Montgomery-product throughput of ONE resident wave per SIMD (the stage kernels' occupancy) as a function of
// how many independent products the wave has in flight at once:
//   call1   the register-ABI call of fp.hpp, one product per call (what the pipeline does today)
//   inl1    the same dependent chain with the product body inlined (no call boundary)
//   inl2/3  two / three independent chains, inlined, so the scheduler can interleave their MADs
//   call2   two independent products in ONE noinline call (56 scalar arguments: beyond the 32 VGPR argument
//           registers of the AMDGPU calling convention -- shows what the stack spill of the rest costs)
//   hipcc -O3 --offload-arch=gfx950 -I include tools/microbench/ilp_rate.hip -o tools/microbench/ilp_rate
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../../lodestar_amd/csrc/tower.hpp"

constexpr int ITERS = 256;

#if defined(__HIP_DEVICE_COMPILE__)
struct fp_ret2 {
  uint32_t l[2 * BLS_NL];
};
__device__ __noinline__ fp_ret2 fp_mul2_r(BLS_PARAMS14(a), BLS_PARAMS14(b), BLS_PARAMS14(c), BLS_PARAMS14(d)) {
  const fp x = BLS_INIT14(a), y = BLS_INIT14(b), z = BLS_INIT14(c), w = BLS_INIT14(d);
  const fp r = fp_mul_body(x, y), s = fp_mul_body(z, w);
  fp_ret2 o;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) {
    o.l[i] = r.l[i];
    o.l[BLS_NL + i] = s.l[i];
  }
  return o;
}
#endif

__device__ __forceinline__ void seed(fp& a, uint32_t t, uint32_t k, uint32_t s) {
  for (int i = 0; i < BLS_NL; i++) a.l[i] = (t * (7919u + 2 * k) + i * (104729u + k) + s) & BLS_MASK;
  a.l[BLS_NL - 1] &= 0xFFFFu;
}
__device__ __forceinline__ void sink(uint32_t* out, const fp& a) {
  uint32_t r = 0;
  for (int i = 0; i < BLS_NL; i++) r ^= a.l[i];
  if (r == 0x1234567u) out[0] = r;
}

__global__ __launch_bounds__(64) void k_call1(uint32_t* out, uint32_t s) {
  fp a, b;
  seed(a, threadIdx.x, 0, s);
  seed(b, threadIdx.x, 1, s);
#pragma unroll 1
  for (int it = 0; it < ITERS; it++) {
    a = fp_mul(a, b);
    b = fp_mul(b, a);
  }
  sink(out, a);
  sink(out, b);
}

__global__ __launch_bounds__(64) void k_inl1(uint32_t* out, uint32_t s) {
  fp a, b;
  seed(a, threadIdx.x, 0, s);
  seed(b, threadIdx.x, 1, s);
#pragma unroll 1
  for (int it = 0; it < ITERS; it++) {
    a = fp_mul_body(a, b);
    b = fp_mul_body(b, a);
  }
  sink(out, a);
  sink(out, b);
}

__global__ __launch_bounds__(64) void k_inl2(uint32_t* out, uint32_t s) {
  fp a, b, c, d;
  seed(a, threadIdx.x, 0, s);
  seed(b, threadIdx.x, 1, s);
  seed(c, threadIdx.x, 2, s);
  seed(d, threadIdx.x, 3, s);
#pragma unroll 1
  for (int it = 0; it < ITERS / 2; it++) {
    a = fp_mul_body(a, b);
    c = fp_mul_body(c, d);
    b = fp_mul_body(b, a);
    d = fp_mul_body(d, c);
  }
  sink(out, a);
  sink(out, b);
  sink(out, c);
  sink(out, d);
}

__global__ __launch_bounds__(64) void k_inl3(uint32_t* out, uint32_t s) {
  fp a, b, c, d, e, f;
  seed(a, threadIdx.x, 0, s);
  seed(b, threadIdx.x, 1, s);
  seed(c, threadIdx.x, 2, s);
  seed(d, threadIdx.x, 3, s);
  seed(e, threadIdx.x, 4, s);
  seed(f, threadIdx.x, 5, s);
#pragma unroll 1
  for (int it = 0; it < ITERS / 3; it++) {
    a = fp_mul_body(a, b);
    c = fp_mul_body(c, d);
    e = fp_mul_body(e, f);
    b = fp_mul_body(b, a);
    d = fp_mul_body(d, c);
    f = fp_mul_body(f, e);
  }
  sink(out, a);
  sink(out, b);
  sink(out, c);
  sink(out, d);
  sink(out, e);
  sink(out, f);
}

__global__ __launch_bounds__(64) void k_call2(uint32_t* out, uint32_t s) {
#if defined(__HIP_DEVICE_COMPILE__)
  fp a, b, c, d;
  seed(a, threadIdx.x, 0, s);
  seed(b, threadIdx.x, 1, s);
  seed(c, threadIdx.x, 2, s);
  seed(d, threadIdx.x, 3, s);
#pragma unroll 1
  for (int it = 0; it < ITERS / 2; it++) {
    fp_ret2 t = fp_mul2_r(BLS_ARGS14(a), BLS_ARGS14(b), BLS_ARGS14(c), BLS_ARGS14(d));
    for (int i = 0; i < BLS_NL; i++) {
      a.l[i] = t.l[i];
      c.l[i] = t.l[BLS_NL + i];
    }
    t = fp_mul2_r(BLS_ARGS14(b), BLS_ARGS14(a), BLS_ARGS14(d), BLS_ARGS14(c));
    for (int i = 0; i < BLS_NL; i++) {
      b.l[i] = t.l[i];
      d.l[i] = t.l[BLS_NL + i];
    }
  }
  sink(out, a);
  sink(out, b);
  sink(out, c);
  sink(out, d);
#endif
}

// code-size probe: the inl2 loop with its body unrolled U times (U x 2 distinct inlined products per
// iteration, ~3.5 KB of code each), to see where instruction fetch starts to cost at 1 wave per SIMD
template <int U>
__device__ __forceinline__ void body_u(fp& a, fp& b, fp& c, fp& d) {
  if constexpr (U > 0) {
    a = fp_mul_body(a, b);
    c = fp_mul_body(c, d);
    b = fp_mul_body(b, a);
    d = fp_mul_body(d, c);
    body_u<U - 1>(a, b, c, d);
  }
}
template <int U>
__global__ __launch_bounds__(64) void k_inl2_u(uint32_t* out, uint32_t s) {
  fp a, b, c, d;
  seed(a, threadIdx.x, 0, s);
  seed(b, threadIdx.x, 1, s);
  seed(c, threadIdx.x, 2, s);
  seed(d, threadIdx.x, 3, s);
#pragma unroll 1
  for (int it = 0; it < ITERS / (2 * U); it++) body_u<U>(a, b, c, d);
  sink(out, a);
  sink(out, b);
  sink(out, c);
  sink(out, d);
}

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

typedef void (*kfn)(uint32_t*, uint32_t);

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int simds = prop.multiProcessorCount * 4;
  uint32_t* d;
  CHECK(hipMalloc(&d, 64));
  struct { const char* name; kfn f; double products_per_lane; } ks[] = {
      {"call1", k_call1, 2.0 * ITERS},
      {"inl1", k_inl1, 2.0 * ITERS},
      {"inl2", k_inl2, 4.0 * (ITERS / 2)},
      {"inl3", k_inl3, 6.0 * (ITERS / 3)},
      {"call2", k_call2, 4.0 * (ITERS / 2)},
      {"inl2_u4 (16 products of code)", k_inl2_u<4>, 4.0 * (ITERS / 2)},
      {"inl2_u16 (64 products of code)", k_inl2_u<16>, 4.0 * (ITERS / 2)},
      {"inl2_u64 (256 products of code)", k_inl2_u<64>, 4.0 * (ITERS / 2)},
  };
  printf("{\"device\": \"%s\", \"simds\": %d, \"results\": [\n", prop.gcnArchName, simds);
  bool first = true;
  for (auto& k : ks) {
    for (int wps : {1, 2, 4}) {
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
      printf("%s  {\"kernel\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"mont_products_per_s\": %.4e}",
             first ? "" : ",\n", k.name, wps, ms / reps, prods / (ms * 1e-3));
      first = false;
    }
  }
  printf("\n]}\n");
  return 0;
}

// What a non-MAD instruction costs beside v_mad_u64_u32 at one wave per SIMD (gfx950): 32 MADs per iteration into
// four independent 64-bit accumulators (carry-out SGPR pairs rotated), interleaved with F independent filler instructions per MAD of one kind --
// v_add_u32, a 64-bit add as v_add_co_u32 + v_addc_co_u32 (counted as two), or v_lshl_add_u64 -- at 1 and 2 waves
// per SIMD.  Prints SIMD cycles per iteration and per MAD as JSON.  Decides whether trading MADs for additions
// (Karatsuba column sums) pays on this issue-bound path.
//   hipcc -O3 --offload-arch=gfx950 tools/microbench/mad_mix.hip -o tools/microbench/mad_mix
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e = (x);                                                           \
    if (e != hipSuccess) {                                                        \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);             \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

constexpr int ITERS = 2048;
constexpr int MADS = 32;

// KIND 0: none, 1: v_add_u32, 2: 64-bit add (v_add_co + v_addc_co), 3: v_lshl_add_u64
template <int KIND, int F>
__global__ __launch_bounds__(64) void k_mix(uint64_t* out, uint32_t s) {
  uint64_t acc[4];
  uint32_t a = threadIdx.x ^ s, b = blockIdx.x + s;
  uint32_t u[8];
  uint64_t w[8];
#pragma unroll
  for (int i = 0; i < 4; i++) acc[i] = a + i;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    u[i] = a * (i + 3);
    w[i] = (uint64_t)b * (i + 5);
  }
#pragma unroll 1
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int j = 0; j < MADS; j++) {
      // carry-out SGPR pairs rotated over four (one shared pair serializes the MADs: the compiler rotates too)
      switch (j & 3) {
        case 0: asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, %0" : "+v"(acc[0]) : "v"(a), "v"(b) : "s40", "s41"); break;
        case 1: asm volatile("v_mad_u64_u32 %0, s[42:43], %1, %2, %0" : "+v"(acc[1]) : "v"(a), "v"(b) : "s42", "s43"); break;
        case 2: asm volatile("v_mad_u64_u32 %0, s[44:45], %1, %2, %0" : "+v"(acc[2]) : "v"(a), "v"(b) : "s44", "s45"); break;
        default: asm volatile("v_mad_u64_u32 %0, s[46:47], %1, %2, %0" : "+v"(acc[3]) : "v"(a), "v"(b) : "s46", "s47"); break;
      }
#pragma unroll
      for (int f = 0; f < F; f++) {
        const int q = (j * F + f) & 7;
        if (KIND == 1) asm volatile("v_add_u32 %0, %0, %1" : "+v"(u[q]) : "v"(b));
        if (KIND == 2)
          asm volatile("v_add_co_u32 %0, vcc, %0, %2\n\tv_addc_co_u32 %1, vcc, %1, %3, vcc"
                       : "+v"(u[q]), "+v"(u[(q + 1) & 7]) : "v"(a), "v"(b) : "vcc");
        if (KIND == 3) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(w[q]) : "v"(w[(q + 3) & 7]));
      }
    }
  }
  uint64_t r = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) r ^= acc[i];
#pragma unroll
  for (int i = 0; i < 8; i++) r ^= u[i] ^ w[i];
  if (r == 0x1234567) out[0] = r;
}

typedef void (*kfn)(uint64_t*, uint32_t);

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int simds = prop.multiProcessorCount * 4;
  uint64_t* d;
  CHECK(hipMalloc(&d, 64));
  struct {
    const char* name;
    int per_mad;
    kfn f;
  } ks[] = {
      {"mad only", 0, k_mix<0, 0>},          {"v_add_u32 x1", 1, k_mix<1, 1>},   {"v_add_u32 x2", 2, k_mix<1, 2>},
      {"add64 (co+addc) x1", 2, k_mix<2, 1>}, {"add64 (co+addc) x2", 4, k_mix<2, 2>},
      {"v_lshl_add_u64 x1", 1, k_mix<3, 1>},  {"v_lshl_add_u64 x2", 2, k_mix<3, 2>},
  };
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  printf("{\"device\": \"%s\", \"simds\": %d, \"clock_khz\": %d, \"mads_per_iter\": %d, \"results\": [\n",
         prop.gcnArchName, simds, prop.clockRate, MADS);
  bool first = true;
  for (auto& k : ks) {
    for (int wps : {1, 2}) {
      const int blocks = simds * wps;
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(64), 0, 0, d, 1u);
      CHECK(hipDeviceSynchronize());
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(64), 0, 0, d, 2u);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      // SIMD cycles per iteration: each SIMD runs wps waves of ITERS iterations
      const double cyc = ms * 1e-3 * prop.clockRate * 1e3 / ((double)ITERS * wps);
      printf("%s {\"variant\": \"%s\", \"fillers_per_mad\": %d, \"waves_per_simd\": %d, \"ms\": %.3f, "
             "\"simd_cycles_per_wave_iter\": %.1f, \"simd_cycles_per_wave_mad\": %.2f}",
             first ? "" : ",\n", k.name, k.per_mad, wps, ms, cyc, cyc / MADS);
      first = false;
    }
  }
  printf("\n]}\n");
  return 0;
}

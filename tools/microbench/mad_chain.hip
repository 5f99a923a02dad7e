// v_mad_u64_u32 dependent-chain latency vs independent accumulators, at 1 and 2 waves per SIMD (gfx950).
// K independent 64-bit accumulators, 32 MADs per iteration in total; the carry-out SGPR pair is either the
// same for every MAD (as the compiler emits) or rotated over four pairs.
//   hipcc -O3 --offload-arch=gfx950 tools/microbench/mad_chain.hip -o tools/microbench/mad_chain
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int ITERS = 4096;
constexpr int PER_ITER = 32;

template <int K, bool ROT>
__global__ __launch_bounds__(64) void k_chain(uint64_t* out, uint32_t s) {
  uint64_t acc[K];
  uint32_t a = threadIdx.x ^ s, b = blockIdx.x + s;
#pragma unroll
  for (int i = 0; i < K; i++) acc[i] = a + i;
#pragma unroll 1
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int j = 0; j < PER_ITER; j++) {
      const int i = j % K;
      if (ROT) {
        switch (j & 3) {
          case 0: asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, %0" : "+v"(acc[i]) : "v"(a), "v"(b) : "s40", "s41"); break;
          case 1: asm volatile("v_mad_u64_u32 %0, s[42:43], %1, %2, %0" : "+v"(acc[i]) : "v"(a), "v"(b) : "s42", "s43"); break;
          case 2: asm volatile("v_mad_u64_u32 %0, s[44:45], %1, %2, %0" : "+v"(acc[i]) : "v"(a), "v"(b) : "s44", "s45"); break;
          default: asm volatile("v_mad_u64_u32 %0, s[46:47], %1, %2, %0" : "+v"(acc[i]) : "v"(a), "v"(b) : "s46", "s47"); break;
        }
      } else {
        asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, %0" : "+v"(acc[i]) : "v"(a), "v"(b) : "s40", "s41");
      }
    }
  }
  uint64_t r = 0;
#pragma unroll
  for (int i = 0; i < K; i++) r ^= acc[i];
  if (r == 0x1234567) out[0] = r;
}

typedef void (*kfn)(uint64_t*, uint32_t);

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int simds = prop.multiProcessorCount * 4;
  uint64_t* d;
  CHECK(hipMalloc(&d, 64));
  struct { const char* name; int k; bool rot; kfn f; } ks[] = {
      {"1 chain", 1, false, k_chain<1, false>},   {"2 chains", 2, false, k_chain<2, false>},
      {"4 chains", 4, false, k_chain<4, false>},  {"8 chains", 8, false, k_chain<8, false>},
      {"1 chain rot", 1, true, k_chain<1, true>}, {"2 chains rot", 2, true, k_chain<2, true>},
      {"4 chains rot", 4, true, k_chain<4, true>}, {"8 chains rot", 8, true, k_chain<8, true>},
  };
  printf("{\"device\": \"%s\", \"simds\": %d, \"clock_khz\": %d, \"results\": [\n", prop.gcnArchName, simds, prop.clockRate);
  bool first = true;
  for (auto& k : ks) {
    for (int wps : {1, 2, 4}) {
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
      const double wave_mads = (double)reps * grid * ITERS * PER_ITER;
      const double simd_cycles = (double)simds * (prop.clockRate * 1e3) * (ms * 1e-3);
      printf("%s  {\"variant\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"lane_mads_per_s\": %.4e, "
             "\"simd_cycles_per_wave_mad\": %.2f}",
             first ? "" : ",\n", k.name, wps, ms / reps, wave_mads * 64 / (ms * 1e-3), simd_cycles / wave_mads);
      first = false;
    }
  }
  printf("\n]}\n");
  return 0;
}

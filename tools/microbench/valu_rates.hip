// VALU integer / fp64 issue-rate microbenchmark for gfx950 (MI355X).
// Measures wave-instructions per cycle per CU for the instructions a 381-bit Montgomery
// multiplication is built from.  The guide (MI355X_MICROARCH.md) does not list integer multiply
// rates; these numbers are the "peak" side of the VALU roofline used in bench.py / DESIGN.md.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int ITERS = 2048;
constexpr int UNROLL = 16;  // instructions per iteration (8 independent chains x 2)

#define BODY8(INS) INS(0) INS(1) INS(2) INS(3) INS(4) INS(5) INS(6) INS(7)

__global__ void k_mad_u64(uint64_t* out, uint32_t s) {
  uint64_t acc[8]; uint32_t a = threadIdx.x ^ s, b = blockIdx.x + s;
  for (int i = 0; i < 8; i++) acc[i] = a + i;
  for (int it = 0; it < ITERS; it++) {
#define INS(i) asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, %0" : "+v"(acc[i]) : "v"(a), "v"(b) : "s40", "s41");
    BODY8(INS) BODY8(INS)
#undef INS
  }
  uint64_t r = 0; for (int i = 0; i < 8; i++) r ^= acc[i];
  if (r == 0x1234567) out[0] = r;
}

__global__ void k_mul_lo(uint64_t* out, uint32_t s) {
  uint32_t acc[8]; uint32_t a = threadIdx.x ^ s;
  for (int i = 0; i < 8; i++) acc[i] = a + i;
  for (int it = 0; it < ITERS; it++) {
#define INS(i) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(acc[i]) : "v"(a));
    BODY8(INS) BODY8(INS)
#undef INS
  }
  uint32_t r = 0; for (int i = 0; i < 8; i++) r ^= acc[i];
  if (r == 0x1234567) out[0] = r;
}

__global__ void k_mul_hi(uint64_t* out, uint32_t s) {
  uint32_t acc[8]; uint32_t a = threadIdx.x ^ s;
  for (int i = 0; i < 8; i++) acc[i] = a + i;
  for (int it = 0; it < ITERS; it++) {
#define INS(i) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(acc[i]) : "v"(a));
    BODY8(INS) BODY8(INS)
#undef INS
  }
  uint32_t r = 0; for (int i = 0; i < 8; i++) r ^= acc[i];
  if (r == 0x1234567) out[0] = r;
}

__global__ void k_mad_u24(uint64_t* out, uint32_t s) {
  uint32_t acc[8]; uint32_t a = threadIdx.x ^ s, b = blockIdx.x;
  for (int i = 0; i < 8; i++) acc[i] = a + i;
  for (int it = 0; it < ITERS; it++) {
#define INS(i) asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(acc[i]) : "v"(a), "v"(b));
    BODY8(INS) BODY8(INS)
#undef INS
  }
  uint32_t r = 0; for (int i = 0; i < 8; i++) r ^= acc[i];
  if (r == 0x1234567) out[0] = r;
}

__global__ void k_addc(uint64_t* out, uint32_t s) {
  uint32_t acc[8]; uint32_t a = threadIdx.x ^ s;
  for (int i = 0; i < 8; i++) acc[i] = a + i;
  for (int it = 0; it < ITERS; it++) {
    // 16 instructions: alternating add_co / addc_co chains through vcc
#define INS(i) asm volatile("v_add_co_u32 %0, vcc, %0, %1\n\tv_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(acc[i]) : "v"(a) : "vcc");
    BODY8(INS)
#undef INS
  }
  uint32_t r = 0; for (int i = 0; i < 8; i++) r ^= acc[i];
  if (r == 0x1234567) out[0] = r;
}

__global__ void k_add_u32(uint64_t* out, uint32_t s) {
  uint32_t acc[8]; uint32_t a = threadIdx.x ^ s;
  for (int i = 0; i < 8; i++) acc[i] = a + i;
  for (int it = 0; it < ITERS; it++) {
#define INS(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(acc[i]) : "v"(a));
    BODY8(INS) BODY8(INS)
#undef INS
  }
  uint32_t r = 0; for (int i = 0; i < 8; i++) r ^= acc[i];
  if (r == 0x1234567) out[0] = r;
}

__global__ void k_lshl_add_u64(uint64_t* out, uint32_t s) {
  uint64_t acc[8]; uint64_t a = threadIdx.x ^ s;
  for (int i = 0; i < 8; i++) acc[i] = a + i;
  for (int it = 0; it < ITERS; it++) {
#define INS(i) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(acc[i]) : "v"(a));
    BODY8(INS) BODY8(INS)
#undef INS
  }
  uint64_t r = 0; for (int i = 0; i < 8; i++) r ^= acc[i];
  if (r == 0x1234567) out[0] = r;
}

__global__ void k_fma_f64(uint64_t* out, uint32_t s) {
  double acc[8]; double a = 1.0 + threadIdx.x * 1e-9, b = 0.999999;
  for (int i = 0; i < 8; i++) acc[i] = a + i;
  for (int it = 0; it < ITERS; it++) {
#define INS(i) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(acc[i]) : "v"(b), "v"(a));
    BODY8(INS) BODY8(INS)
#undef INS
  }
  double r = 0; for (int i = 0; i < 8; i++) r += acc[i];
  if (r == 1234567.0) out[0] = 1;
}

__global__ void k_cndmask(uint64_t* out, uint32_t s) {
  uint32_t acc[8]; uint32_t a = threadIdx.x ^ s;
  for (int i = 0; i < 8; i++) acc[i] = a + i;
  for (int it = 0; it < ITERS; it++) {
#define INS(i) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(acc[i]) : "v"(a) : "vcc");
    BODY8(INS) BODY8(INS)
#undef INS
  }
  uint32_t r = 0; for (int i = 0; i < 8; i++) r ^= acc[i];
  if (r == 0x1234567) out[0] = r;
}

typedef void (*kfn)(uint64_t*, uint32_t);

int main() {
  hipDeviceProp_t prop; CHECK(hipGetDeviceProperties(&prop, 0));
  int cus = prop.multiProcessorCount;
  printf("{\"device\": \"%s\", \"cus\": %d, \"clock_khz\": %d, \"results\": [\n", prop.gcnArchName, cus, prop.clockRate);
  uint64_t* d; CHECK(hipMalloc(&d, 64));
  struct { const char* name; kfn f; } ks[] = {
    {"v_mad_u64_u32", k_mad_u64}, {"v_mul_lo_u32", k_mul_lo}, {"v_mul_hi_u32", k_mul_hi},
    {"v_mad_u32_u24", k_mad_u24}, {"v_add_co_u32+v_addc_co_u32", k_addc}, {"v_add_u32", k_add_u32},
    {"v_lshl_add_u64", k_lshl_add_u64}, {"v_fma_f64", k_fma_f64}, {"v_cndmask_b32", k_cndmask},
  };
  int nk = sizeof(ks) / sizeof(ks[0]);
  int block = 256;
  for (int occ = 0; occ < 2; occ++) {
    int blocks_per_cu = occ == 0 ? 8 : 1;  // 32 waves/CU vs 4 waves/CU (1 per SIMD)
    int grid = cus * blocks_per_cu;
    for (int i = 0; i < nk; i++) {
      hipLaunchKernelGGL(ks[i].f, dim3(grid), dim3(block), 0, 0, d, 1u);  // warmup
      CHECK(hipDeviceSynchronize());
      hipEvent_t e0, e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
      CHECK(hipEventRecord(e0));
      const int reps = 5;
      for (int r = 0; r < reps; r++) hipLaunchKernelGGL(ks[i].f, dim3(grid), dim3(block), 0, 0, d, (uint32_t)r);
      CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
      float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
      double wave_instr = (double)reps * grid * (block / 64) * ITERS * UNROLL;
      double lane_ops_per_s = wave_instr * 64 / (ms * 1e-3);
      double wave_instr_per_cu_per_ns = wave_instr / cus / (ms * 1e6);
      printf("  {\"instr\": \"%s\", \"waves_per_cu\": %d, \"ms\": %.3f, \"lane_ops_per_s\": %.4e, \"wave_instr_per_cu_per_ns\": %.4f}%s\n",
             ks[i].name, blocks_per_cu * 4, ms / reps, lane_ops_per_s, wave_instr_per_cu_per_ns,
             (occ == 1 && i == nk - 1) ? "" : ",");
    }
  }
  printf("]}\n");
  return 0;
}

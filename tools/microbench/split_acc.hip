// Montgomery-product throughput as a register-ABI call chain (the pipeline's form) for two column schedules:
//   cur    fp.hpp's product scanning: ONE 64-bit accumulator per column, so every v_mad_u64_u32 of a product
//          depends on the one before it (392 serial MADs per multiplication)
//   split  per column k the a*b terms and the m_i*p terms of i < k-1 form a chain that does not depend on column
//          k-1 (only on m_{k-2}); the carry of column k-1, m_{k-1}*p_1, m_k and m_k*p_0 are the only serial steps
//          -- one extra 64-bit add per column, a critical path of ~5 instructions per column
// for fp_mul (one lane), fp_sqr and the lane-pair dot product (fp2x.hpp), at 1 / 2 / 4 waves per SIMD, and checks
// that both schedules give identical limbs.
//   hipcc -O3 --offload-arch=gfx950 tools/microbench/split_acc.hip -o tools/microbench/split_acc
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../../lodestar_amd/csrc/fp2x.hpp"

constexpr int ITERS = 256;

// ---- split-schedule bodies ----
// Column k's products go alternately into two accumulators (two independent MAD chains a wave can issue back to back
// where one chain waits ~11 cycles per MAD); an empty asm on each partial sum keeps LLVM's reassociation from folding
// them back into one chain.  m_{k-1} p_1 and m_k p_0 stay on the serial carry path.
#if defined(__HIP_DEVICE_COMPILE__)
#define OPAQUE64(x) asm("" : "+v"(x))
#else
#define OPAQUE64(x) ((void)0)
#endif
struct acc2 {
  uint64_t t[2] = {0, 0};
  int n = 0;
  BLS_INL void mad(uint32_t x, uint32_t y) {
    t[n & 1] += (uint64_t)x * y;
    n++;
  }
  BLS_INL uint64_t sum(uint64_t carry) {
    OPAQUE64(t[0]);
    OPAQUE64(t[1]);
    return t[0] + t[1] + carry;
  }
};
template <int KIND, bool GATE>  // KIND 0 mul, 1 sqr, 2 dot; GATE: column k's chains start after column k-2's carry
BLS_INL fp split_body(const fp& x1, const fp& y1, const fp& x2, const fp& y2) {
  fp r;
  uint32_t m[BLS_NL], a2[BLS_NL];
  if (KIND == 1) {
#pragma unroll
    for (int i = 0; i < BLS_NL; i++) a2[i] = x1.l[i] << 1;
  }
  uint64_t carry = 0;
  uint32_t gate[2 * BLS_NL];
#pragma unroll
  for (int k = 0; k < 2 * BLS_NL - 1; k++) {
    const int lo = k < BLS_NL ? 0 : k - BLS_NL + 1, hi = k < BLS_NL ? k : BLS_NL - 1;
    acc2 t;
#if defined(__HIP_DEVICE_COMPILE__)
    if (GATE && k >= 2) asm("" : "+v"(t.t[0]), "+v"(t.t[1]) : "v"(gate[k - 2]));
#endif
    if (KIND == 1) {
#pragma unroll
      for (int i = lo; 2 * i < k; i++) t.mad(a2[i], x1.l[k - i]);
      if ((k & 1) == 0) t.mad(x1.l[k >> 1], x1.l[k >> 1]);
    } else {
#pragma unroll
      for (int i = lo; i <= hi; i++) {
        t.mad(x1.l[i], y1.l[k - i]);
        if (KIND == 2) t.mad(x2.l[i], y2.l[k - i]);
      }
    }
    const int mhi = k < BLS_NL ? k - 1 : BLS_NL - 1;  // m_i p_{k-i} for i in [lo, mhi]
#pragma unroll
    for (int i = lo; i < mhi; i++) t.mad(m[i], FP_P.l[k - i]);
    uint64_t acc = t.sum(carry);
    if (mhi >= lo) acc += (uint64_t)m[mhi] * FP_P.l[k - mhi];
    if (k < BLS_NL) {
      const uint32_t q = ((uint32_t)acc * BLS_N0INV) & BLS_MASK;
      m[k] = q;
      acc += (uint64_t)q * FP_P.l[0];
    } else {
      r.l[k - BLS_NL] = (uint32_t)acc & BLS_MASK;
    }
    carry = acc >> BLS_LB;
    gate[k] = (uint32_t)carry;
  }
  r.l[BLS_NL - 1] = (uint32_t)carry;
  return r;
}

#if defined(__HIP_DEVICE_COMPILE__)
// ---- register-ABI wrappers: V = 0 cur, 1 split ----
#define RET14(r)                                         \
  {                                                      \
    const fp r_ = r;                                     \
    fp_ret o;                                            \
    for (int i = 0; i < BLS_NL; i++) o.l[i] = r_.l[i]; \
    return o;                                            \
  }
template <int V>
__device__ __noinline__ fp_ret mul_r(BLS_PARAMS14(a), BLS_PARAMS14(b)) {
  const fp x = BLS_INIT14(a), y = BLS_INIT14(b);
  if (V == 0) { RET14(fp_mul_body(x, y)) }
  RET14((split_body<0, V == 2>(x, y, x, y)))
}
template <int V>
__device__ __noinline__ fp_ret sqr_r(BLS_PARAMS14(a)) {
  const fp x = BLS_INIT14(a);
  if (V == 0) { RET14(fp_sqr_body(x)) }
  RET14((split_body<1, V == 2>(x, x, x, x)))
}
// the lane-pair product: this lane's coefficient (fp2x_mul_body's operand setup, then the dot product)
template <int V>
__device__ __noinline__ fp_ret pair_r(BLS_PARAMS14(a_), BLS_PARAMS14(b_)) {
  const fp a = BLS_INIT14(a_), b = BLS_INIT14(b_);
  const bool odd = fp2x_k() != 0;
  fp pa, b0, y;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) {
    pa.l[i] = dpp_swap(a.l[i]);
    b0.l[i] = dpp_even(b.l[i]);
    const uint32_t b1 = dpp_odd(b.l[i]);
    y.l[i] = odd ? b1 : FP_16P_K.l[i] - b1;
  }
  if (V == 0) { RET14(fp_dot_body(a, b0, pa, y)) }
  RET14((split_body<2, V == 2>(a, b0, pa, y)))
}

template <int OP, int V>
__device__ __forceinline__ fp call(const fp& a, const fp& b) {
  fp_ret t;
  if (OP == 0) t = mul_r<V>(BLS_ARGS14(a), BLS_ARGS14(b));
  if (OP == 1) t = sqr_r<V>(BLS_ARGS14(a));
  if (OP == 2) t = pair_r<V>(BLS_ARGS14(a), BLS_ARGS14(b));
  fp r;
  for (int i = 0; i < BLS_NL; i++) r.l[i] = t.l[i];
  return r;
}
#else
template <int OP, int V>
__device__ fp call(const fp& a, const fp&) { return a; }  // host pass: never runs
#endif

__device__ __forceinline__ void seed(fp& a, uint32_t t, uint32_t k, uint32_t s) {
  for (int i = 0; i < BLS_NL; i++) a.l[i] = (t * (7919u + 2 * k) + i * (104729u + k) + s * 31337u) & BLS_MASK;
  a.l[BLS_NL - 1] &= 0xFFFFu;
}

// dependent chain a = a.b; b = b.a (sqr: a = a^2; b = b^2 + ... keeps two chains like the mul form)
template <int OP, int V>
__global__ __launch_bounds__(64) void k_chain(uint32_t* out, uint32_t s, int iters) {
  fp a, b;
  seed(a, blockIdx.x * 64 + threadIdx.x, 0, s);
  seed(b, blockIdx.x * 64 + threadIdx.x, 1, s);
#pragma unroll 1
  for (int it = 0; it < iters; it++) {
    a = call<OP, V>(a, b);
    b = call<OP, V>(b, a);
  }
  const uint32_t g = blockIdx.x * 64 + threadIdx.x;
  for (int i = 0; i < BLS_NL; i++) {
    out[(2 * i) * gridDim.x * 64 + g] = a.l[i];
    out[(2 * i + 1) * gridDim.x * 64 + g] = b.l[i];
  }
}

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
typedef void (*kfn)(uint32_t*, uint32_t, int);

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int simds = prop.multiProcessorCount * 4;
  const size_t words = (size_t)simds * 4 * 64 * 2 * BLS_NL;
  uint32_t *d0, *d1;
  CHECK(hipMalloc(&d0, words * 4));
  CHECK(hipMalloc(&d1, words * 4));
  uint32_t* h0 = (uint32_t*)malloc(words * 4);
  uint32_t* h1 = (uint32_t*)malloc(words * 4);
  struct { const char* name; kfn v[3]; } ks[] = {
      {"fp_mul", {k_chain<0, 0>, k_chain<0, 1>, k_chain<0, 2>}},
      {"fp_sqr", {k_chain<1, 0>, k_chain<1, 1>, k_chain<1, 2>}},
      {"fp2x_mul (lane pair)", {k_chain<2, 0>, k_chain<2, 1>, k_chain<2, 2>}},
  };
  printf("{\"device\": \"%s\", \"simds\": %d, \"calls_per_lane\": %d, \"results\": [\n", prop.gcnArchName, simds,
         2 * ITERS);
  bool first = true;
  for (auto& k : ks) {
    for (int wps : {1, 2, 4}) {
      const int grid = simds * wps;
      float ms[3];
      size_t diff[3] = {0, 0, 0};
      for (int v = 0; v < 3; v++) {
        kfn f = k.v[v];
        uint32_t* d = v ? d1 : d0;
        hipLaunchKernelGGL(f, dim3(grid), dim3(64), 0, 0, d, 1u, ITERS);
        CHECK(hipDeviceSynchronize());
        hipEvent_t e0, e1;
        CHECK(hipEventCreate(&e0));
        CHECK(hipEventCreate(&e1));
        CHECK(hipEventRecord(e0));
        const int reps = 3;
        for (int r = 0; r < reps; r++) hipLaunchKernelGGL(f, dim3(grid), dim3(64), 0, 0, d, 1u, ITERS);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipEventElapsedTime(&ms[v], e0, e1));
        ms[v] /= reps;
        const size_t n = (size_t)grid * 64 * 2 * BLS_NL;
        CHECK(hipMemcpy(v ? h1 : h0, d, n * 4, hipMemcpyDeviceToHost));
        if (v)
          for (size_t i = 0; i < n; i++) diff[v] += h0[i] != h1[i];
      }
      const double calls = 2.0 * ITERS * grid * 64;
      printf("%s  {\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": {\"cur\": %.3f, \"split\": %.3f, \"gated\": %.3f}, "
             "\"products_per_s\": {\"cur\": %.4e, \"split\": %.4e, \"gated\": %.4e}, \"limb_mismatches\": [%zu, %zu]}",
             first ? "" : ",\n", k.name, wps, ms[0], ms[1], ms[2], calls / (ms[0] * 1e-3), calls / (ms[1] * 1e-3),
             calls / (ms[2] * 1e-3), diff[1], diff[2]);
      first = false;
    }
  }
  printf("\n]}\n");
  return 0;
}

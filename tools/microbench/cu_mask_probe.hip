// CU-mask probe (round 6): where do the workgroups of a stream created by hipExtStreamCreateWithCUMask run, and how
// long does a small kernel on a CU partition wait while the rest of the chip is busy?
//
// Step 1 (safe under any bit -> CU mapping): mask bits {33 k, k = 0..7}.  Whether the driver deals mask bits
// round-robin over the 8 XCDs (bit i -> XCD i % 8) or in blocks of 32 CUs (bit i -> XCD i / 32), these bits give one CU
// on every XCD, so no workgroup can be dealt to an XCD without CUs.  The two mappings put those CUs on different shader
// engines (interleaved: within-XCD index 33k / 8 = 0, 4, 8, ... -> all on SE 0; blocked: index k -> SE k % 4), which the
// workgroups' HW_ID tells apart.  Only when the interleaved mapping is confirmed does step 2 use bits 0..7 / 0..15.
// Step 3: a long "hog" kernel on a stream masked to the complement, then the latency of a 1-workgroup kernel on the
// partition stream, on a high-priority unmasked stream and on a normal unmasked stream.
// Prints one JSON object.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/microbench/cu_mask_probe.hip -o tools/microbench/cu_mask_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <unistd.h>

#include <set>
#include <vector>

#define CHECK(x)                                                                                 \
  do {                                                                                           \
    hipError_t e_ = (x);                                                                         \
    if (e_ != hipSuccess) {                                                                      \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);     \
      return 1;                                                                                  \
    }                                                                                            \
  } while (0)

// per workgroup: XCC_ID, HW_ID (raw); the lanes spin `iters` dependent VALU steps so the workgroups overlap in time
__global__ void k_where(uint32_t* out, uint32_t iters, uint32_t* sink) {
  uint32_t xcc, hw;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  uint32_t v = threadIdx.x + 1;
  for (uint32_t i = 0; i < iters; i++) v = v * 1664525u + 1013904223u;
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = xcc;
    out[2 * blockIdx.x + 1] = hw;
  }
  if (v == 0x12345678u) sink[0] = v;
}

struct Where {
  uint32_t xcc, se, cu, sh;
};

static std::vector<Where> run_where(hipStream_t st, uint32_t nblk, uint32_t iters, uint32_t* d_out, uint32_t* d_sink,
                                    bool& ok) {
  std::vector<uint32_t> h(2 * nblk);
  hipLaunchKernelGGL(k_where, dim3(nblk), dim3(64), 0, st, d_out, iters, d_sink);
  ok = hipGetLastError() == hipSuccess;
  ok = ok && hipStreamSynchronize(st) == hipSuccess;
  ok = ok && hipMemcpy(h.data(), d_out, 8 * nblk, hipMemcpyDeviceToHost) == hipSuccess;
  std::vector<Where> w(nblk);
  for (uint32_t b = 0; b < nblk; b++) {
    const uint32_t hw = h[2 * b + 1];
    w[b] = {h[2 * b], (hw >> 13) & 7, (hw >> 8) & 15, (hw >> 12) & 1};
  }
  return w;
}

static void print_where(const char* name, const std::vector<Where>& w) {
  std::set<uint32_t> cus;
  for (auto& x : w) cus.insert(x.xcc << 16 | x.se << 8 | x.sh << 4 | x.cu);
  printf("\"%s\": {\"distinct_cus\": %zu, \"cus\": [", name, cus.size());
  bool first = true;
  for (uint32_t c : cus) {
    printf("%s[%u, %u, %u, %u]", first ? "" : ", ", c >> 16, (c >> 8) & 255, (c >> 4) & 15, c & 15);
    first = false;
  }
  printf("]}, ");
}

static std::vector<uint32_t> mask_of(const std::vector<int>& bits, bool complement, int n_cu) {
  std::vector<uint32_t> m((n_cu + 31) / 32, 0);
  for (int b : bits) m[b / 32] |= 1u << (b % 32);
  if (complement)
    for (int i = 0; i < n_cu; i++) m[i / 32] ^= 1u << (i % 32);
  return m;
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int n_cu = prop.multiProcessorCount;
  uint32_t *d_out, *d_sink;
  CHECK(hipMalloc(&d_out, 8 * 4096));
  CHECK(hipMalloc(&d_sink, 4));
  printf("{\"n_cu\": %d, ", n_cu);
  bool ok;
  // step 0: unmasked
  hipStream_t s0;
  CHECK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  auto w0 = run_where(s0, 1024, 20000, d_out, d_sink, ok);
  if (!ok) return 1;
  print_where("unmasked_1024wg", w0);
  // step 1: bits {33k}
  std::vector<int> b33;
  for (int k = 0; k < 8; k++) b33.push_back(33 * k);
  auto m33 = mask_of(b33, false, n_cu);
  hipStream_t s33;
  CHECK(hipExtStreamCreateWithCUMask(&s33, (uint32_t)m33.size(), m33.data()));
  auto w33 = run_where(s33, 64, 20000, d_out, d_sink, ok);
  if (!ok) return 1;
  print_where("mask_33k_64wg", w33);
  // interleaved mapping confirmed: one CU per XCD, all on SE 0, 8 distinct XCDs
  std::set<uint32_t> xccs, ses, cus;
  for (auto& x : w33) {
    xccs.insert(x.xcc);
    ses.insert(x.se);
    cus.insert(x.xcc << 16 | x.se << 8 | x.sh << 4 | x.cu);
  }
  const bool interleaved = xccs.size() == 8 && cus.size() == 8 && ses.size() == 1 && *ses.begin() == 0;
  printf("\"interleaved\": %s, ", interleaved ? "true" : "false");
  if (!interleaved) {
    printf("\"stopped\": \"mapping not confirmed\"}\n");
    return 0;
  }
  // step 2: contiguous bit ranges
  for (int nb : {8, 16}) {
    std::vector<int> bits;
    for (int i = 0; i < nb; i++) bits.push_back(i);
    auto m = mask_of(bits, false, n_cu);
    hipStream_t s;
    CHECK(hipExtStreamCreateWithCUMask(&s, (uint32_t)m.size(), m.data()));
    auto w = run_where(s, 128, 20000, d_out, d_sink, ok);
    if (!ok) return 1;
    char name[64];
    snprintf(name, sizeof name, "mask_bits0_%d_128wg", nb - 1);
    print_where(name, w);
    auto mc = mask_of(bits, true, n_cu);
    hipStream_t sc;
    CHECK(hipExtStreamCreateWithCUMask(&sc, (uint32_t)mc.size(), mc.data()));
    auto wc = run_where(sc, 2048, 20000, d_out, d_sink, ok);
    if (!ok) return 1;
    // the complement must never touch the partition
    std::set<uint32_t> part;
    for (auto& x : w) part.insert(x.xcc << 16 | x.se << 8 | x.sh << 4 | x.cu);
    int overlap = 0;
    std::set<uint32_t> cc;
    for (auto& x : wc) {
      const uint32_t key = x.xcc << 16 | x.se << 8 | x.sh << 4 | x.cu;
      cc.insert(key);
      overlap += part.count(key) ? 1 : 0;
    }
    printf("\"complement_of_bits0_%d\": {\"distinct_cus\": %zu, \"workgroups_on_partition\": %d}, ", nb - 1, cc.size(),
           overlap);
    CHECK(hipStreamDestroy(s));
    CHECK(hipStreamDestroy(sc));
  }
  // step 3: latency of a 1-workgroup kernel while a hog fills the chip (the hog on the complement of bits 0..7)
  {
    std::vector<int> bits;
    for (int i = 0; i < 8; i++) bits.push_back(i);
    auto mp = mask_of(bits, false, n_cu), mc = mask_of(bits, true, n_cu);
    hipStream_t sp, sc, shi, snorm;
    CHECK(hipExtStreamCreateWithCUMask(&sp, (uint32_t)mp.size(), mp.data()));
    CHECK(hipExtStreamCreateWithCUMask(&sc, (uint32_t)mc.size(), mc.data()));
    int lo, hi;
    CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    CHECK(hipStreamCreateWithPriority(&shi, hipStreamNonBlocking, hi));
    CHECK(hipStreamCreateWithPriority(&snorm, hipStreamNonBlocking, lo));
    hipStream_t hog_unmasked;
    CHECK(hipStreamCreateWithFlags(&hog_unmasked, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    uint32_t* d_hog;
    CHECK(hipMalloc(&d_hog, 8 * 65536));
    auto timed = [&](hipStream_t st, float& ms) -> bool {
      if (hipEventRecord(e0, st) != hipSuccess) return false;
      hipLaunchKernelGGL(k_where, dim3(1), dim3(64), 0, st, d_out, 20000u, d_sink);
      if (hipEventRecord(e1, st) != hipSuccess) return false;
      if (hipEventSynchronize(e1) != hipSuccess) return false;
      return hipEventElapsedTime(&ms, e0, e1) == hipSuccess;
    };
    float idle_ms = 0;
    if (!timed(sp, idle_ms)) return 1;
    if (!timed(sp, idle_ms)) return 1;
    printf("\"small_kernel_idle_ms\": %.4f, ", idle_ms);
    const char* names[3] = {"partition_stream", "high_priority_unmasked", "normal_unmasked"};
    hipStream_t sts[3] = {sp, shi, snorm};
    for (int masked_hog = 1; masked_hog >= 0; masked_hog--) {
      printf("\"%s\": {", masked_hog ? "hog_on_complement" : "hog_unmasked");
      for (int k = 0; k < 3; k++) {
        // hog: 16384 one-wave workgroups of ~2-3 ms each, several per SIMD
        hipStream_t hs = masked_hog ? sc : hog_unmasked;
        hipLaunchKernelGGL(k_where, dim3(16384), dim3(64), 0, hs, d_hog, 4000000u, d_sink);
        if (hipGetLastError() != hipSuccess) return 1;
        // let it fill the chip
        hipEvent_t eh;
        CHECK(hipEventCreate(&eh));
        CHECK(hipEventRecord(eh, hs));
        usleep(20000);
        float ms = -1;
        if (!timed(sts[k], ms)) return 1;
        const bool hog_running = hipEventQuery(eh) == hipErrorNotReady;
        CHECK(hipStreamSynchronize(hs));
        CHECK(hipEventDestroy(eh));
        printf("%s\"%s\": {\"ms\": %.4f, \"hog_still_running\": %s}", k ? ", " : "", names[k], ms,
               hog_running ? "true" : "false");
      }
      printf("}%s", masked_hog ? ", " : "");
    }
  }
  printf("}\n");
  return 0;
}

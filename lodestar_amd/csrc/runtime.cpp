// Host runtime of libblsgpu: the C ABI declared in include/blsgpu.h.
//
// Replaces BlsMultiThreadWorkerPool's job plumbing (reference packages/beacon-node/src/chain/bls/
// multithread/index.ts:134-412) and the worker's batch/fallback policy (multithread/worker.ts:32-108)
// with HIP streams on MI355X and no worker threads doing arithmetic:
//   * jobs are sharded across devices in contiguous, cost-balanced ranges (never splitting a job);
//   * each device owns several "slots" (a HIP stream + its staging and work buffers).  A call takes one
//     free slot per device it uses, so independent verifySignatureSets calls run concurrently on the
//     GPU -- the way the reference keeps all its workers busy -- and the device is filled by several
//     batches' lane-per-set kernels at once;
//   * each shard runs the stage kernels (k_*.hip): signature decode + subgroup check, hash_to_G2,
//     pubkey aggregation, r_i scaling, per-set Miller loops, then the batch-group tail;
//   * batchable jobs are packed into groups of >= group_sets sets (random linear combination, one final
//     exponentiation per group); non-batchable jobs are their own group; a single-set non-batchable
//     job uses r = 1 (= CoreVerify, maybeBatch.ts:34-38);
//   * a failed group with several clean jobs is split into <= 8 contiguous sub-ranges that are re-checked
//     with the same group kernels (k-ary bisection) until every job is resolved on its own.  The per-set
//     Miller loops stay on the device, so a re-check costs one Miller loop + final exponentiation.
//     Per job the answer is the reference's: valid iff every set of the job verifies (worker.ts:76-98).
// There is no CPU verification path: without a usable GPU blsgpu_init fails.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
#include <sys/random.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/blsgpu.h"
#include "kernels.h"

namespace {

struct HipError {
  hipError_t e;
};
#define HIPCHK(x)                             \
  do {                                        \
    hipError_t _e = (x);                      \
    if (_e != hipSuccess) throw HipError{_e}; \
  } while (0)

template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t cap = 0;
  void ensure(size_t n) {
    if (n <= cap) return;
    if (p) HIPCHK(hipFree(p));
    p = nullptr;
    size_t c = std::max<size_t>(n, cap * 3 / 2);
    HIPCHK(hipMalloc((void**)&p, c * sizeof(T)));
    cap = c;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

template <class T>
struct HostBuf {  // pinned staging
  T* p = nullptr;
  size_t cap = 0;
  void ensure(size_t n) {
    if (n <= cap) return;
    if (p) HIPCHK(hipHostFree(p));
    p = nullptr;
    size_t c = std::max<size_t>(n, cap * 3 / 2);
    HIPCHK(hipHostMalloc((void**)&p, c * sizeof(T), hipHostMallocDefault));
    cap = c;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
};

constexpr int kStages = 8;
constexpr size_t kMillerLineWords = 68 * 6 * W_FP;  // MILLER_STEPS x (l0, c1, c4) per set (k_miller.hip)

// One in-flight batch on one device: a stream and every per-call buffer.
struct Slot {
  hipStream_t stream = nullptr;
  hipEvent_t ev[kStages + 1] = {};
  // d_in / h_in: every per-call input packed into one arena (one H2D transfer); d_res / h_res: job errors +
  // group verdicts (one D2H transfer).  Each transfer is a blit kernel that must find a free SIMD among
  // the full-register-file verification waves, so a batch pays for each one in queueing delay.
  DevBuf<uint8_t> d_in, d_res, d_flags, d_ok, d_include;
  DevBuf<int8_t> d_status;
  DevBuf<uint32_t> d_ranges, d_work, d_S, d_F, d_lines;
  HostBuf<uint8_t> h_in, h_res, h_ok;
  HostBuf<uint32_t> h_ranges;

  void release_all() {
    d_in.release(); d_res.release(); d_flags.release(); d_ok.release(); d_include.release(); d_status.release();
    d_ranges.release(); d_work.release(); d_S.release(); d_F.release(); d_lines.release();
    h_in.release(); h_res.release(); h_ok.release(); h_ranges.release();
  }
};

struct Device {
  int id = 0;
  hipStream_t table_stream = nullptr;
  // pubkey table (AoS, W_PKTAB words per key): verification holds it shared, uploads exclusive
  std::shared_mutex table_mu;
  DevBuf<uint32_t> table;
  uint32_t table_n = 0;
  // slots
  std::mutex slot_mu;
  std::condition_variable slot_cv;
  std::vector<Slot*> slots;
  std::vector<Slot*> free_slots;

  void add_slot() {
    Slot* s = new Slot();
    HIPCHK(hipSetDevice(id));
    HIPCHK(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
    for (auto& e : s->ev) HIPCHK(hipEventCreate(&e));
    slots.push_back(s);
    free_slots.push_back(s);
  }
  Slot* acquire() {
    std::unique_lock<std::mutex> lk(slot_mu);
    slot_cv.wait(lk, [&] { return !free_slots.empty(); });
    Slot* s = free_slots.back();
    free_slots.pop_back();
    return s;
  }
  void release(Slot* s) {
    {
      std::lock_guard<std::mutex> lk(slot_mu);
      free_slots.push_back(s);
    }
    slot_cv.notify_one();
  }
  void destroy_all() {
    (void)hipSetDevice(id);
    for (Slot* s : slots) {
      if (s->stream) (void)hipStreamSynchronize(s->stream);
      s->release_all();
      for (auto& e : s->ev)
        if (e) (void)hipEventDestroy(e);
      if (s->stream) (void)hipStreamDestroy(s->stream);
      delete s;
    }
    slots.clear();
    free_slots.clear();
    table.release();
    if (table_stream) (void)hipStreamDestroy(table_stream);
  }
};

inline uint64_t splitmix64_at(uint64_t seed, uint64_t i) {
  // i-th output of the SplitMix64 stream seeded with `seed` (counter form: state_i = seed + (i+1) gamma)
  uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z = z ^ (z >> 31);
  return z ? z : 1;
}

}  // namespace

struct blsgpu_ctx {
  std::vector<Device*> devs;
  std::atomic<bool> closed{false};
  std::atomic<int> inflight{0};
  std::mutex async_mu;
  std::condition_variable async_cv;
  std::mutex table_mu;
  std::mutex opt_mu;
  int64_t group_sets = 256;
  int64_t max_devices = 64;
  int64_t split_ways = 8;
  bool profile = false;
};

namespace {

struct Shard {
  uint32_t job_begin, job_end;  // job range
  uint32_t set_begin, set_end;  // set range
};

// Runs one device's shard on one slot.  Writes job_result[job_begin..job_end).
int run_shard(blsgpu_ctx* ctx, Device& d, Slot& sl, const blsgpu_batch& b, const Shard& sh, int8_t* job_result,
              uint64_t seed, blsgpu_stats& st) {
  const uint32_t n = sh.set_end - sh.set_begin;
  const uint32_t nj = sh.job_end - sh.job_begin;
  if (nj == 0) return BLSGPU_OK;
  HIPCHK(hipSetDevice(d.id));
  const uint32_t s0 = sh.set_begin;
  const uint32_t stride = std::max<uint32_t>(n, 1);
  const uint32_t split_ways = (uint32_t)std::max<int64_t>(2, ctx->split_ways);

  // ---- host-side job structure: groups (contiguous job ranges), scalars ------------------------
  // Non-batchable jobs are groups of their own; consecutive batchable jobs are packed until a group
  // holds >= group_sets sets.  Empty jobs get no group (rejected with EMPTY_SET).
  // Input arena layout (256-B aligned sections; groups <= jobs bounds the ranges section):
  //   scalars n*8 | job_first_set (nj+1)*4 | sigs n*192 | sig_len n*4 | msgs n*32 | ranges nj*8 |
  //   table mode: set_pk_first (n+1)*4, pk_index npk*4;  bytes mode: pk_bytes n*96
  const bool table_mode = b.pk_bytes == nullptr;
  const uint32_t npk = table_mode ? b.set_pk_first[sh.set_end] - b.set_pk_first[s0] : 0;
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t o_scal = 0, o_jobs = al(o_scal + (size_t)n * 8), o_sigs = al(o_jobs + (size_t)(nj + 1) * 4),
               o_siglen = al(o_sigs + (size_t)n * 192), o_msgs = al(o_siglen + (size_t)n * 4),
               o_ranges = al(o_msgs + (size_t)n * 32), o_pk = al(o_ranges + (size_t)nj * 8),
               o_pkidx = al(o_pk + (size_t)(n + 1) * 4),
               in_bytes = table_mode ? o_pkidx + (size_t)npk * 4 : o_pk + (size_t)n * 96;
  sl.h_in.ensure(in_bytes);
  sl.d_in.ensure(in_bytes);
  uint8_t* const hin = sl.h_in.p;
  uint64_t* scal = reinterpret_cast<uint64_t*>(hin + o_scal);
  uint32_t* hjobs = reinterpret_cast<uint32_t*>(hin + o_jobs);
  std::vector<uint32_t> job_group(nj, UINT32_MAX);
  std::vector<std::pair<uint32_t, uint32_t>> group_jobs;  // [first job, end job) (shard-relative)
  {
    uint32_t cur_sets = 0;
    bool open = false;
    for (uint32_t j = 0; j < nj; j++) {
      const uint32_t gj = sh.job_begin + j;
      const uint32_t a = b.job_first_set[gj] - s0, e = b.job_first_set[gj + 1] - s0;
      hjobs[j] = a;
      const bool batchable = b.job_flags && (b.job_flags[gj] & 1u);
      if (e == a) {
        open = false;
        continue;
      }
      if (!batchable) {
        job_group[j] = (uint32_t)group_jobs.size();
        group_jobs.push_back({j, j + 1});
        // single-set non-batchable job: CoreVerify (r = 1); multi-set: random linear combination
        for (uint32_t i = a; i < e; i++) scal[i] = (e - a == 1) ? 1ull : splitmix64_at(seed, s0 + i);
        open = false;
        continue;
      }
      for (uint32_t i = a; i < e; i++) scal[i] = splitmix64_at(seed, s0 + i);
      if (!open || cur_sets >= (uint32_t)ctx->group_sets) {
        group_jobs.push_back({j, j});
        cur_sets = 0;
        open = true;
      }
      job_group[j] = (uint32_t)group_jobs.size() - 1;
      group_jobs.back().second = j + 1;
      cur_sets += e - a;
    }
    hjobs[nj] = n;
  }
  auto job_sets = [&](uint32_t j) {
    const uint32_t gj = sh.job_begin + j;
    return std::make_pair(b.job_first_set[gj] - s0, b.job_first_set[gj + 1] - s0);
  };

  // ---- stage inputs in the pinned arena and copy it to the device in one transfer ----------------
  const uint32_t sstride = b.sig_stride;
  uint8_t* hsigs = hin + o_sigs;
  uint32_t* hsiglen = reinterpret_cast<uint32_t*>(hin + o_siglen);
  for (uint32_t i = 0; i < n; i++) {
    uint32_t len = b.sig_len[s0 + i];
    uint32_t cl = (len == 96 || len == 192) ? len : 0;
    memcpy(hsigs + (size_t)i * 192, b.sigs + (size_t)(s0 + i) * sstride, cl);
    hsiglen[i] = len;
  }
  memcpy(hin + o_msgs, b.msgs + (size_t)s0 * 32, (size_t)n * 32);
  if (table_mode) {
    uint32_t* hpkfirst = reinterpret_cast<uint32_t*>(hin + o_pk);
    const uint32_t base = b.set_pk_first[s0];
    for (uint32_t i = 0; i <= n; i++) hpkfirst[i] = b.set_pk_first[s0 + i] - base;
    memcpy(hin + o_pkidx, b.pk_index + base, (size_t)npk * 4);
  } else {
    memcpy(hin + o_pk, b.pk_bytes + (size_t)s0 * 96, (size_t)n * 96);
  }
  const uint32_t ng0 = (uint32_t)group_jobs.size();
  const uint32_t max_ranges = std::max<uint32_t>(std::max(ng0, nj), 1);
  uint32_t* hranges = reinterpret_cast<uint32_t*>(hin + o_ranges);
  for (uint32_t g = 0; g < ng0; g++) {
    hranges[2 * g] = job_sets(group_jobs[g].first).first;
    hranges[2 * g + 1] = job_sets(group_jobs[g].second - 1).second;
  }

  sl.d_flags.ensure((size_t)stride * 2);
  sl.d_status.ensure((size_t)stride * 2);
  sl.d_include.ensure(stride);
  const size_t o_ok = al(nj), res_bytes = o_ok + max_ranges;
  sl.d_res.ensure(res_bytes);
  sl.h_res.ensure(res_bytes);
  sl.d_S.ensure((size_t)W_G2J * max_ranges);
  sl.d_F.ensure((size_t)W_FP12 * max_ranges);
  // work area: sig_aff, h_aff, pk_jac, pk_aff, rsig, f
  const size_t work_words = (size_t)stride * (W_G2A + W_G2A + W_G1J + W_G1A + W_G2J + W_FP12);
  sl.d_work.ensure(work_words);
  sl.d_lines.ensure((size_t)stride * kMillerLineWords);
  hipStream_t s = sl.stream;
  uint8_t* const din = sl.d_in.p;
  HIPCHK(hipMemcpyAsync(din, hin, in_bytes, hipMemcpyHostToDevice, s));
  uint8_t* const d_ok0 = sl.d_res.p + o_ok;

  PipelineBuffers pb;
  pb.n = stride;
  pb.sigs = din + o_sigs;
  pb.sig_len = reinterpret_cast<uint32_t*>(din + o_siglen);
  pb.sig_stride = 192;
  pb.msgs = din + o_msgs;
  pb.pk_bytes = table_mode ? nullptr : din + o_pk;
  pb.set_pk_first = table_mode ? reinterpret_cast<uint32_t*>(din + o_pk) : nullptr;
  pb.pk_index = table_mode ? reinterpret_cast<uint32_t*>(din + o_pkidx) : nullptr;
  pb.pk_table = d.table.p;
  pb.pk_table_n = d.table_n;
  pb.scalars = reinterpret_cast<uint64_t*>(din + o_scal);
  pb.job_first_set = reinterpret_cast<uint32_t*>(din + o_jobs);
  pb.n_jobs = nj;
  uint32_t* w = sl.d_work.p;
  pb.sig_aff = w; w += (size_t)stride * W_G2A;
  pb.h_aff = w; w += (size_t)stride * W_G2A;
  pb.pk_jac = w; w += (size_t)stride * W_G1J;
  pb.pk_aff = w; w += (size_t)stride * W_G1A;
  pb.rsig = w; w += (size_t)stride * W_G2J;
  pb.f = w;
  pb.lines = sl.d_lines.p;
  pb.flags = sl.d_flags.p;
  pb.status = sl.d_status.p;
  pb.job_err = reinterpret_cast<int8_t*>(sl.d_res.p);
  pb.include = sl.d_include.p;

  // ---- kernel pipeline ---------------------------------------------------------------------------
  const bool prof = ctx->profile;
  auto mark = [&](int k) {
    if (prof) HIPCHK(hipEventRecord(sl.ev[k], s));
  };
  mark(0);
  launch_sig_decode(pb, n, s);
  mark(1);
  launch_hash_to_g2(pb, n, s);
  mark(2);
  if (table_mode) launch_pk_aggregate(pb, n, s);
  mark(3);
  launch_pk_finish(pb, n, s);
  mark(4);
  launch_sig_scale(pb, n, s);
  mark(5);
  launch_miller_sets(pb, n, s);
  launch_job_mask(pb, s);
  mark(6);
  launch_group_reduce(pb, reinterpret_cast<uint32_t*>(din + o_ranges), ng0, sl.d_S.p, sl.d_F.p, s);
  mark(7);
  launch_group_check(sl.d_S.p, sl.d_F.p, ng0, d_ok0, s);
  mark(8);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(sl.h_res.p, sl.d_res.p, o_ok + ng0, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  st.groups += ng0;
  if (prof) {
    for (int k = 0; k < kStages; k++) {
      float ms = 0;
      HIPCHK(hipEventElapsedTime(&ms, sl.ev[k], sl.ev[k + 1]));
      st.stage_ms[k] += ms;
    }
  }

  // ---- per-job results ---------------------------------------------------------------------------
  std::vector<int> jr(nj, 0);
  for (uint32_t j = 0; j < nj; j++) {
    const int err = (int8_t)sl.h_res.p[j];
    jr[j] = err ? -err : 2;  // 2 = pending
  }
  // pending work: lists of clean jobs whose batch equation failed
  std::vector<std::vector<uint32_t>> failed;
  for (uint32_t g = 0; g < ng0; g++) {
    std::vector<uint32_t> clean;
    for (uint32_t j = group_jobs[g].first; j < group_jobs[g].second; j++)
      if (jr[j] == 2) clean.push_back(j);
    if (clean.empty()) continue;
    if (sl.h_res.p[o_ok + g]) {
      for (uint32_t j : clean) jr[j] = 1;
      if (group_jobs[g].second - group_jobs[g].first > 1)
        for (uint32_t j : clean) st.batch_sigs_success += job_sets(j).second - job_sets(j).first;
    } else if (clean.size() == 1) {
      jr[clean[0]] = 0;
    } else {
      st.batch_retries++;
      failed.push_back(std::move(clean));
    }
  }

  // ---- fallback: k-ary bisection of failed groups -------------------------------------------------
  while (!failed.empty()) {
    std::vector<std::vector<uint32_t>> parts;
    for (auto& jobs : failed) {
      const size_t k = std::min<size_t>(split_ways, jobs.size());
      for (size_t p = 0; p < k; p++) {
        size_t lo = jobs.size() * p / k, hi = jobs.size() * (p + 1) / k;
        if (hi > lo) parts.emplace_back(jobs.begin() + lo, jobs.begin() + hi);
      }
    }
    const uint32_t np = (uint32_t)parts.size();
    sl.h_ranges.ensure(2 * np);
    sl.d_ranges.ensure(2 * np);
    sl.d_ok.ensure(np);
    sl.h_ok.ensure(np);
    sl.d_S.ensure((size_t)W_G2J * np);
    sl.d_F.ensure((size_t)W_FP12 * np);
    for (uint32_t q = 0; q < np; q++) {
      sl.h_ranges.p[2 * q] = job_sets(parts[q].front()).first;
      sl.h_ranges.p[2 * q + 1] = job_sets(parts[q].back()).second;
    }
    // Sub-ranges may span error jobs between clean ones; their sets are masked out on the device.  A
    // single-job part covers exactly its own sets, so every final `false` is decided on the job alone.
    HIPCHK(hipMemcpyAsync(sl.d_ranges.p, sl.h_ranges.p, (size_t)np * 8, hipMemcpyHostToDevice, s));
    launch_group_reduce(pb, sl.d_ranges.p, np, sl.d_S.p, sl.d_F.p, s);
    launch_group_check(sl.d_S.p, sl.d_F.p, np, sl.d_ok.p, s);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(sl.h_ok.p, sl.d_ok.p, np, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    std::vector<std::vector<uint32_t>> next;
    for (uint32_t q = 0; q < np; q++) {
      if (sl.h_ok.p[q]) {
        for (uint32_t j : parts[q]) jr[j] = 1;
      } else if (parts[q].size() == 1) {
        jr[parts[q][0]] = 0;
      } else {
        next.push_back(std::move(parts[q]));
      }
    }
    failed.swap(next);
  }
  for (uint32_t j = 0; j < nj; j++) job_result[sh.job_begin + j] = (int8_t)jr[j];
  return BLSGPU_OK;
}

int validate_batch(const blsgpu_ctx* ctx, const blsgpu_batch* b) {
  if (!b || !b->job_first_set) return BLSGPU_ERR_ARGS;
  if (b->n_jobs == 0) return BLSGPU_OK;
  if (b->job_first_set[0] != 0 || b->job_first_set[b->n_jobs] != b->n_sets) return BLSGPU_ERR_ARGS;
  for (uint32_t j = 0; j < b->n_jobs; j++)
    if (b->job_first_set[j + 1] < b->job_first_set[j]) return BLSGPU_ERR_ARGS;
  if (b->n_sets == 0) return BLSGPU_OK;
  if (!b->msgs || !b->sigs || !b->sig_len) return BLSGPU_ERR_ARGS;
  if (b->sig_stride < 96) return BLSGPU_ERR_ARGS;
  for (uint32_t i = 0; i < b->n_sets; i++)
    if (b->sig_len[i] > b->sig_stride && (b->sig_len[i] == 96 || b->sig_len[i] == 192)) return BLSGPU_ERR_ARGS;
  if (!b->pk_bytes) {
    if (!b->set_pk_first || !b->pk_index) return BLSGPU_ERR_ARGS;
    if (b->set_pk_first[0] != 0) return BLSGPU_ERR_ARGS;
    for (uint32_t i = 0; i < b->n_sets; i++)
      if (b->set_pk_first[i + 1] < b->set_pk_first[i]) return BLSGPU_ERR_ARGS;
    uint32_t tn = ctx->devs.empty() ? 0 : ctx->devs[0]->table_n;
    for (uint32_t k = 0; k < b->set_pk_first[b->n_sets]; k++)
      if (b->pk_index[k] >= tn) return BLSGPU_ERR_ARGS;
  }
  return BLSGPU_OK;
}

}  // namespace

extern "C" {

int blsgpu_init(const int* devices, int n_devices, blsgpu_ctx** out) {
  if (!out) return BLSGPU_ERR_ARGS;
  *out = nullptr;
  // Slots need hardware queues of their own: kernels of streams that share one run in order, so a batch's
  // long single-batch tail (k_group_check) blocks the next batch's stage kernels.  HIP's default (and the
  // usual environment) is 4 queues per process; on MI355X 8 measured 1.70M vs 1.32M sets/s on C2 with 12
  // slots, and 16 fails queue creation (HSA_STATUS_ERROR_OUT_OF_RESOURCES) -- profiles/r01_hwq.json.  So a
  // setting below 8 is raised to 8 (BLSGPU_KEEP_HW_QUEUES=1 keeps it).  HIP reads it once, at its
  // initialization, so this only takes effect when blsgpu_init is the process's first HIP call.
  {
    const char* q = getenv("GPU_MAX_HW_QUEUES");
    const char* keep = getenv("BLSGPU_KEEP_HW_QUEUES");
    if (!(keep && keep[0] == '1') && (!q || atoi(q) < 8)) setenv("GPU_MAX_HW_QUEUES", "8", 1);
  }
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return BLSGPU_ERR_NO_DEVICE;
  std::vector<int> ids;
  if (devices && n_devices > 0) {
    for (int i = 0; i < n_devices; i++) {
      if (devices[i] < 0 || devices[i] >= count) return BLSGPU_ERR_ARGS;
      ids.push_back(devices[i]);
    }
  } else {
    for (int i = 0; i < count; i++) ids.push_back(i);
  }
  blsgpu_ctx* ctx = new blsgpu_ctx();
  try {
    for (int id : ids) {
      Device* d = new Device();
      d->id = id;
      ctx->devs.push_back(d);
      HIPCHK(hipSetDevice(id));
      HIPCHK(hipStreamCreateWithFlags(&d->table_stream, hipStreamNonBlocking));
      for (int k = 0; k < 4; k++) d->add_slot();
    }
  } catch (HipError&) {
    blsgpu_destroy(ctx);
    return BLSGPU_ERR_NO_DEVICE;
  }
  *out = ctx;
  return BLSGPU_OK;
}

void blsgpu_destroy(blsgpu_ctx* ctx) {
  if (!ctx) return;
  ctx->closed = true;
  {
    std::unique_lock<std::mutex> lk(ctx->async_mu);
    ctx->async_cv.wait(lk, [&] { return ctx->inflight.load() == 0; });
  }
  for (Device* d : ctx->devs) {
    // wait until no synchronous caller holds a slot
    {
      std::unique_lock<std::mutex> lk(d->slot_mu);
      d->slot_cv.wait(lk, [&] { return d->free_slots.size() == d->slots.size(); });
    }
    d->destroy_all();
    delete d;
  }
  delete ctx;
}

int blsgpu_device_count(const blsgpu_ctx* ctx) { return ctx ? (int)ctx->devs.size() : 0; }

uint32_t blsgpu_pubkeys_count(const blsgpu_ctx* ctx) {
  return (ctx && !ctx->devs.empty()) ? ctx->devs[0]->table_n : 0;
}

int blsgpu_pubkeys_upload(blsgpu_ctx* ctx, uint32_t first_index, const uint8_t* pk96, uint32_t n) {
  if (!ctx) return BLSGPU_ERR_ARGS;
  if (ctx->closed) return BLSGPU_ERR_CLOSED;
  if (n == 0) return BLSGPU_OK;
  if (!pk96) return BLSGPU_ERR_ARGS;
  std::lock_guard<std::mutex> tl(ctx->table_mu);
  int result = BLSGPU_OK;
  try {
    for (Device* d : ctx->devs) {
      std::unique_lock<std::shared_mutex> lk(d->table_mu);
      HIPCHK(hipSetDevice(d->id));
      hipStream_t ts = d->table_stream;
      const uint32_t need = first_index + n;
      uint8_t* dpk = nullptr;
      int8_t* dst = nullptr;
      uint32_t* tmp = nullptr;
      HIPCHK(hipMalloc((void**)&dpk, (size_t)n * 96));
      HIPCHK(hipMalloc((void**)&dst, n));
      HIPCHK(hipMalloc((void**)&tmp, (size_t)n * W_PKTAB * 4));
      HIPCHK(hipMemcpyAsync(dpk, pk96, (size_t)n * 96, hipMemcpyHostToDevice, ts));
      launch_pk_table_fill(dpk, n, tmp, dst, ts);
      HIPCHK(hipGetLastError());
      std::vector<int8_t> hst(n);
      HIPCHK(hipMemcpyAsync(hst.data(), dst, n, hipMemcpyDeviceToHost, ts));
      HIPCHK(hipStreamSynchronize(ts));
      int err = 0;
      for (uint32_t i = 0; i < n && !err; i++) err = hst[i];
      if (!err) {
        if (need > d->table.cap / W_PKTAB) {
          DevBuf<uint32_t> nt;
          nt.ensure((size_t)std::max<uint32_t>(need, d->table_n + d->table_n / 2) * W_PKTAB);
          if (d->table_n)
            HIPCHK(hipMemcpy(nt.p, d->table.p, (size_t)d->table_n * W_PKTAB * 4, hipMemcpyDeviceToDevice));
          d->table.release();
          d->table = nt;
        }
        HIPCHK(hipMemcpy(d->table.p + (size_t)first_index * W_PKTAB, tmp, (size_t)n * W_PKTAB * 4,
                         hipMemcpyDeviceToDevice));
        d->table_n = std::max(d->table_n, need);
      }
      (void)hipFree(dpk);
      (void)hipFree(dst);
      (void)hipFree(tmp);
      if (err) {
        result = err;
        break;
      }
    }
  } catch (HipError&) {
    return BLSGPU_DEVICE_ERROR;
  }
  return result;
}

int blsgpu_set_option(blsgpu_ctx* ctx, const char* key, int64_t value) {
  if (!ctx || !key) return BLSGPU_ERR_ARGS;
  std::string k(key);
  std::lock_guard<std::mutex> lk(ctx->opt_mu);
  if (k == "group_sets") {
    if (value < 1) return BLSGPU_ERR_ARGS;
    ctx->group_sets = value;
  } else if (k == "profile") {
    ctx->profile = value != 0;
  } else if (k == "max_devices") {
    if (value < 1) return BLSGPU_ERR_ARGS;
    ctx->max_devices = value;
  } else if (k == "split_ways") {
    if (value < 2) return BLSGPU_ERR_ARGS;
    ctx->split_ways = value;
  } else if (k == "slots") {
    if (value < 1 || value > 64) return BLSGPU_ERR_ARGS;
    try {
      for (Device* d : ctx->devs) {
        std::lock_guard<std::mutex> sl(d->slot_mu);
        while ((int64_t)d->slots.size() < value) d->add_slot();
      }
    } catch (HipError&) {
      return BLSGPU_DEVICE_ERROR;
    }
  } else {
    return BLSGPU_ERR_ARGS;
  }
  return BLSGPU_OK;
}

int blsgpu_verify(blsgpu_ctx* ctx, const blsgpu_batch* b, int8_t* job_result, blsgpu_stats* stats) {
  if (!ctx) return BLSGPU_ERR_ARGS;
  if (ctx->closed) return BLSGPU_ERR_CLOSED;
  int v = validate_batch(ctx, b);
  if (v) return v;
  if (b->n_jobs && !job_result) return BLSGPU_ERR_ARGS;
  blsgpu_stats local{};
  uint64_t seed = b->seed;
  if (seed == 0) {
    while (seed == 0) {
      if (getrandom(&seed, sizeof(seed), 0) != (ssize_t)sizeof(seed)) return BLSGPU_ERR_ARGS;
    }
  }
  // cost-balanced contiguous sharding of jobs over devices
  const uint32_t nd_all = (uint32_t)std::min<int64_t>((int64_t)ctx->devs.size(), ctx->max_devices);
  const uint32_t nd = std::max<uint32_t>(1, std::min<uint32_t>(nd_all, (b->n_sets + 255) / 256));
  std::vector<double> cost(b->n_jobs + 1, 0.0);
  for (uint32_t j = 0; j < b->n_jobs; j++) {
    double c = 0;
    for (uint32_t i = b->job_first_set[j]; i < b->job_first_set[j + 1]; i++) {
      c += 1.0;
      if (!b->pk_bytes) c += (b->set_pk_first[i + 1] - b->set_pk_first[i]) / 256.0;
    }
    cost[j + 1] = cost[j] + c;
  }
  std::vector<Shard> shards;
  uint32_t j0 = 0;
  for (uint32_t k = 0; k < nd; k++) {
    double target = cost[b->n_jobs] * (k + 1) / nd;
    uint32_t j1 = j0;
    if (k + 1 == nd) {
      j1 = b->n_jobs;
    } else {
      while (j1 < b->n_jobs && cost[j1 + 1] <= target) j1++;
    }
    shards.push_back({j0, j1, b->job_first_set[j0], b->job_first_set[j1]});
    j0 = j1;
  }
  auto t0 = std::chrono::steady_clock::now();
  std::vector<blsgpu_stats> sst(shards.size());
  std::vector<int> rc(shards.size(), BLSGPU_OK);
  auto work = [&](size_t k) {
    Device& d = *ctx->devs[k];
    std::shared_lock<std::shared_mutex> tl(d.table_mu);
    Slot* sl = d.acquire();
    try {
      rc[k] = run_shard(ctx, d, *sl, *b, shards[k], job_result, seed, sst[k]);
    } catch (HipError&) {
      rc[k] = BLSGPU_DEVICE_ERROR;
    } catch (...) {
      rc[k] = BLSGPU_DEVICE_ERROR;
    }
    d.release(sl);
    if (rc[k] == BLSGPU_DEVICE_ERROR)
      for (uint32_t j = shards[k].job_begin; j < shards[k].job_end; j++) job_result[j] = -BLSGPU_DEVICE_ERROR;
  };
  if (shards.size() == 1) {
    work(0);
  } else {
    std::vector<std::thread> th;
    for (size_t k = 0; k < shards.size(); k++) th.emplace_back(work, k);
    for (auto& t : th) t.join();
  }
  auto t1 = std::chrono::steady_clock::now();
  int status = BLSGPU_OK;
  for (int k = 0; k < kStages; k++) local.stage_ms[k] = sst[0].stage_ms[k];
  for (size_t k = 0; k < shards.size(); k++) {
    local.groups += sst[k].groups;
    local.batch_retries += sst[k].batch_retries;
    local.batch_sigs_success += sst[k].batch_sigs_success;
    if (rc[k] != BLSGPU_OK) status = rc[k];
  }
  local.devices_used = (uint32_t)shards.size();
  local.device_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
  if (stats) *stats = local;
  return status == BLSGPU_DEVICE_ERROR ? BLSGPU_OK : status;  // device errors are reported per job
}

int blsgpu_submit(blsgpu_ctx* ctx, const blsgpu_batch* b, int8_t* job_result, blsgpu_stats* stats,
                  blsgpu_done_cb done, void* user) {
  if (!ctx || !b) return BLSGPU_ERR_ARGS;
  if (ctx->closed) return BLSGPU_ERR_CLOSED;
  int v = validate_batch(ctx, b);
  if (v) return v;
  // deep-copy the inputs so the caller may reuse its buffers immediately
  struct Owned {
    blsgpu_batch b;
    std::vector<uint32_t> jfs, siglen, pkfirst, pkidx;
    std::vector<uint8_t> jflags, pkb, msgs, sigs;
  };
  Owned* o = new Owned();
  o->b = *b;
  o->jfs.assign(b->job_first_set, b->job_first_set + b->n_jobs + 1);
  o->b.job_first_set = o->jfs.data();
  if (b->job_flags) {
    o->jflags.assign(b->job_flags, b->job_flags + b->n_jobs);
    o->b.job_flags = o->jflags.data();
  }
  o->siglen.assign(b->sig_len, b->sig_len + b->n_sets);
  o->b.sig_len = o->siglen.data();
  o->sigs.assign(b->sigs, b->sigs + (size_t)b->n_sets * b->sig_stride);
  o->b.sigs = o->sigs.data();
  o->msgs.assign(b->msgs, b->msgs + (size_t)b->n_sets * 32);
  o->b.msgs = o->msgs.data();
  if (b->pk_bytes) {
    o->pkb.assign(b->pk_bytes, b->pk_bytes + (size_t)b->n_sets * 96);
    o->b.pk_bytes = o->pkb.data();
  } else {
    o->pkfirst.assign(b->set_pk_first, b->set_pk_first + b->n_sets + 1);
    o->pkidx.assign(b->pk_index, b->pk_index + b->set_pk_first[b->n_sets]);
    o->b.set_pk_first = o->pkfirst.data();
    o->b.pk_index = o->pkidx.data();
  }
  {
    std::lock_guard<std::mutex> lk(ctx->async_mu);
    ctx->inflight++;
  }
  std::thread([ctx, o, job_result, stats, done, user]() {
    int rc = ctx->closed ? BLSGPU_ERR_CLOSED : blsgpu_verify(ctx, &o->b, job_result, stats);
    delete o;
    if (done) done(user, rc);
    {
      std::lock_guard<std::mutex> lk(ctx->async_mu);
      ctx->inflight--;
    }
    ctx->async_cv.notify_all();
  }).detach();
  return BLSGPU_OK;
}

const char* blsgpu_code_name(int code) {
  switch (code) {
    case BLSGPU_OK: return "BLST_SUCCESS";
    case BLSGPU_BAD_ENCODING: return "BLST_BAD_ENCODING";
    case BLSGPU_POINT_NOT_ON_CURVE: return "BLST_POINT_NOT_ON_CURVE";
    case BLSGPU_POINT_NOT_IN_GROUP: return "BLST_POINT_NOT_IN_GROUP";
    case BLSGPU_AGGR_TYPE_MISMATCH: return "BLST_AGGR_TYPE_MISMATCH";
    case BLSGPU_VERIFY_FAIL: return "BLST_VERIFY_FAIL";
    case BLSGPU_PK_IS_INFINITY: return "BLST_PK_IS_INFINITY";
    case BLSGPU_BAD_SCALAR: return "BLST_BAD_SCALAR";
    case BLSGPU_INVALID_SIZE: return "BLST_INVALID_SIZE";
    case BLSGPU_EMPTY_AGGREGATE: return "EMPTY_AGGREGATE_ARRAY";
    case BLSGPU_EMPTY_SET: return "Empty signature set";
    case BLSGPU_DEVICE_ERROR: return "BLSGPU_DEVICE_ERROR";
    case BLSGPU_ERR_ARGS: return "BLSGPU_ERR_ARGS";
    case BLSGPU_ERR_NO_DEVICE: return "BLSGPU_ERR_NO_DEVICE";
    case BLSGPU_ERR_CLOSED: return "QUEUE_ERROR_QUEUE_ABORTED";
    default: return nullptr;
  }
}

int blsgpu_debug_op(blsgpu_ctx* ctx, int op, uint32_t n, const uint8_t* in, uint32_t in_stride, uint8_t* out,
                    uint32_t out_stride, int32_t* status) {
  if (!ctx || ctx->devs.empty() || !in || !out || !status) return BLSGPU_ERR_ARGS;
  if (n == 0) return BLSGPU_OK;
  Device* d = ctx->devs[0];
  Slot* sl = d->acquire();
  uint8_t *din = nullptr, *dout = nullptr;
  int32_t* dst = nullptr;
  int rc = BLSGPU_OK;
  try {
    HIPCHK(hipSetDevice(d->id));
    HIPCHK(hipMalloc((void**)&din, (size_t)n * in_stride));
    HIPCHK(hipMalloc((void**)&dout, (size_t)n * out_stride));
    HIPCHK(hipMalloc((void**)&dst, (size_t)n * 4));
    HIPCHK(hipMemcpy(din, in, (size_t)n * in_stride, hipMemcpyHostToDevice));
    HIPCHK(hipMemset(dout, 0, (size_t)n * out_stride));
    launch_debug_op(op, n, din, in_stride, dout, out_stride, dst, sl->stream);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(sl->stream));
    HIPCHK(hipMemcpy(out, dout, (size_t)n * out_stride, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(status, dst, (size_t)n * 4, hipMemcpyDeviceToHost));
  } catch (HipError&) {
    rc = BLSGPU_DEVICE_ERROR;
  }
  if (din) (void)hipFree(din);
  if (dout) (void)hipFree(dout);
  if (dst) (void)hipFree(dst);
  d->release(sl);
  return rc;
}

}  // extern "C"

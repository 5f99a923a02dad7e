// Launchers for the verification-pipeline kernels (k_*.hip), called by runtime.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Word counts of the SoA records (element i, word w at base[w * stride + i])
#define W_FP 14
#define W_G1A (2 * W_FP)
#define W_G1J (3 * W_FP)
#define W_G2A (4 * W_FP)
#define W_G2J (6 * W_FP)
#define W_FP12 (12 * W_FP)
// Pubkey table entries: AoS, 32 words (x limbs, y limbs, pad) = one 128-byte line per key
#define W_PKTAB 32

// set flags (uint8 per set)
#define SF_SIG_INF 1u
#define SF_H_INF 2u
#define SF_PK_INF 4u

struct PipelineBuffers {
  uint32_t n;  // SoA stride (>= n_sets)
  // inputs
  const uint8_t* sigs;
  const uint32_t* sig_len;
  uint32_t sig_stride;
  const uint8_t* msgs;
  const uint8_t* pk_bytes;       // bytes mode or nullptr
  const uint32_t* set_pk_first;  // table mode
  const uint32_t* pk_index;
  const uint32_t* pk_table;  // AoS W_PKTAB words per key
  uint32_t pk_table_n;
  const uint64_t* scalars;
  const uint32_t* job_first_set;  // [n_jobs + 1], shard-relative
  uint32_t n_jobs;
  // intermediates
  uint32_t* sig_aff;  // W_G2A
  uint32_t* h_aff;    // W_G2A
  uint32_t* pk_jac;   // W_G1J (table mode aggregate)
  uint32_t* pk_aff;   // W_G1A (r * pk)
  uint32_t* rsig;     // W_G2J
  uint32_t* f;        // W_FP12
  uint32_t* lines;    // Miller lines: MILLER_STEPS x 3 Fp2 (6 * W_FP words) per set, step-major SoA
  uint8_t* flags;     // [2n]: sig flags, hash flags
  int8_t* status;     // [2n]: signature status, pubkey status
  int8_t* job_err;    // [n_jobs]: first pubkey/signature error of the job (0 = clean)
  uint8_t* include;   // [n]: set belongs to a clean job (enters the batch equation)
};

void launch_sig_decode(const PipelineBuffers& b, uint32_t n_sets, hipStream_t s);
void launch_hash_to_g2(const PipelineBuffers& b, uint32_t n_sets, hipStream_t s);
void launch_pk_aggregate(const PipelineBuffers& b, uint32_t n_sets, hipStream_t s);
void launch_pk_finish(const PipelineBuffers& b, uint32_t n_sets, hipStream_t s);
void launch_sig_scale(const PipelineBuffers& b, uint32_t n_sets, hipStream_t s);
void launch_miller_sets(const PipelineBuffers& b, uint32_t n_sets, hipStream_t s);
// per-job error status and the per-set include mask of the batch equation
void launch_job_mask(const PipelineBuffers& b, hipStream_t s);
// Batch groups: group g covers sets [ranges[2g], ranges[2g+1]) (only included sets count).
// reduce: S_g = sum r_i sig_i (W_G2J SoA, stride n_groups), F_g = prod f_i (W_FP12 SoA, stride n_groups)
void launch_group_reduce(const PipelineBuffers& b, const uint32_t* ranges, uint32_t n_groups, uint32_t* S,
                         uint32_t* F, hipStream_t s);
// check: ok_g = FinalExp(F_g * MillerLoop(-g1, S_g)) == 1
void launch_group_check(const uint32_t* S, const uint32_t* F, uint32_t n_groups, uint8_t* ok, hipStream_t s);
// pubkey table upload: decode 96-byte affine encodings into table entries, per-entry status
void launch_pk_table_fill(const uint8_t* pk96, uint32_t n, uint32_t* table_dst, int8_t* status, hipStream_t s);
// debug ops (blsgpu_debug_op)
void launch_debug_op(int op, uint32_t n, const uint8_t* in, uint32_t in_stride, uint8_t* out, uint32_t out_stride,
                     int32_t* status, hipStream_t s);

// Launchers for the verification-pipeline kernels (k_*.hip), called by runtime.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <vector>

// Word counts of the SoA records (element i, word w at base[w * stride + i])
#define W_FP 14
#define W_G1A (2 * W_FP)
#define W_G1J (3 * W_FP)
#define W_G2A (4 * W_FP)
#define W_G2J (6 * W_FP)
#define W_FP12 (12 * W_FP)
// Pubkey table entries: AoS, 32 words (x limbs, y limbs, pad) = one 128-byte line per key
#define W_PKTAB 32
// Miller-loop line coefficients per message: 68 steps x (l0, c1, c4)
#define MILLER_STEPS 68
#define W_LINE (3 * 2 * W_FP)

// set flags (uint8 per set)
#define SF_SIG_INF 1u
// per-message flags
#define MF_H_INF 1u

struct PipelineBuffers {
  uint32_t n;  // SoA stride of per-set arrays (>= n_sets)
  // ---- inputs
  const uint8_t* sigs;
  const uint32_t* sig_len;
  uint32_t sig_stride;
  // public keys: pk_bytes && !set_pk_first: one 96-B key per set; pk_bytes && set_pk_first: set i aggregates
  // keys [set_pk_first[i], set_pk_first[i+1]) of pk_bytes; !pk_bytes: table entries pk_index[...]
  const uint8_t* pk_bytes;
  const uint32_t* set_pk_first;
  const uint32_t* pk_index;
  const uint32_t* pk_table;  // AoS W_PKTAB words per key
  uint32_t pk_table_n;
  // aggregation list: k_pk_aggregate runs one wave per set agg_sets[0 .. n_agg) (all sets when null); with
  // pk_direct1, a set of exactly one key skips it and k_pk_finish reads / decodes that key itself
  const uint32_t* agg_sets;
  uint32_t n_agg;
  uint32_t pk_direct1;
  const uint64_t* scalars;  // batch scalar words (k_common.hpp jac_mul_scalar_word), 0 = r = 1
  uint32_t* scal_tab;       // signed-window tables: 8 x W_G2J words per set (SoA, stride n)
  const uint32_t* job_first_set;  // [n_jobs + 1], shard-relative
  uint32_t n_jobs;
  // messages, deduplicated per call: set i signs umsgs[msg_idx[i]]
  const uint8_t* umsgs;
  const uint32_t* msg_idx;
  uint32_t n_umsg;
  uint32_t nm;  // SoA stride of per-message arrays (>= n_umsg)
  // pairing units (same-message merging): unit u = the included sets unit_sets[unit_set_first[u] ..
  // unit_set_first[u+1]) of one batch group, all signing umsgs[unit_msg[u]]; P_u = sum r_i pk_i
  uint32_t n_units;
  const uint32_t* unit_set_first;
  const uint32_t* unit_sets;
  const uint32_t* unit_msg;
  // ---- intermediates
  uint32_t* sig_aff;  // W_G2A, per set
  uint32_t* h_aff;    // W_G2A, per message
  uint32_t* h_jac;    // W_G2J, per message: H(m) before the batched affine conversion (k_inv.hip)
  uint32_t* h_norm;   // W_FP, per message: N(d) of the hash prep, then N(z) of h_jac
  uint32_t* h_prep;   // 7 x W_FP2, per message: the hash_to_G2 state across its batched inversion (k_hash.hip)
  uint32_t* h_q;      // 2 x W_G2J, per message: the two mapped points iso3(SSWU(u_j)) (stride 2 nm, k_hash.hip)
  uint32_t* inv_buf;     // W_FP, per max(set, message): batch inversion output of the message branch (k_inv.hip)
  uint32_t* inv_buf_pk;  // W_FP, per set: the pubkey branch's (the two branches run on different streams)
  uint32_t* pk_jac;   // W_G1J, per set (aggregate)
  uint32_t* pk_aff;   // W_G1A, per set (r * pk, affine)
  uint32_t* rsig;     // W_G2J, per set
  uint32_t* unit_p;   // W_G1A, per unit (stride n)
  // Miller chunks: chunk c multiplies the Miller values of items chunk_items[chunk_first[c] ..
  // chunk_first[c+1]) (sets, or units) into ONE accumulator with shared squarings -> f_chunk[c]
  uint32_t n_chunks;
  const uint32_t* chunk_first;
  const uint32_t* chunk_items;
  uint32_t* f_chunk;  // W_FP12, per chunk (stride n)
  uint32_t* lines;    // Miller lines, per message: MILLER_STEPS x W_LINE words, step-major SoA (stride nm)
  uint8_t* flags;     // [n]: sig flags
  uint8_t* mflags;    // [nm]: message flags
  uint8_t* unit_ok;   // [n]: unit has a finite P_u
  int8_t* status;     // [3n]: signature status, pubkey status, aggregation status
  int8_t* job_err;    // [n_jobs]: first pubkey/signature error of the job (0 = clean)
  uint8_t* include;   // [n]: set belongs to a clean job (enters the batch equation)
};

// coop: small and mid-size runs -- the [|z|] chains (subgroup check, cofactor clearing) as cooperative 16-lane
// doublings (g2_coop.hpp), for latency; exclusive: each cooperative workgroup takes a CU to itself (small runs only:
// beyond ~one workgroup per CU the padding serializes the launch)
// (decoded: recorded after the decode, before the small-run subgroup checks)
void launch_sig_decode(const PipelineBuffers& b, uint32_t n_sets, hipStream_t s, bool coop = false,
                       hipEvent_t decoded = nullptr, bool exclusive = true);
// spec[i] = the signature of set i decoded (the speculative MSM's include mask)
void launch_spec_mask(const PipelineBuffers& b, uint32_t n_sets, uint8_t* spec, hipStream_t s);
void launch_hash_prep(const PipelineBuffers& b, hipStream_t s);
void launch_hash_map(const PipelineBuffers& b, const uint32_t* inv, hipStream_t s);
void launch_hash_to_g2(const PipelineBuffers& b, hipStream_t s, bool coop = false,
                       bool exclusive = true);  // over the unique messages
void launch_pk_aggregate(const PipelineBuffers& b, uint32_t n_sets, hipStream_t s);
void launch_pk_finish(const PipelineBuffers& b, uint32_t n_sets, hipStream_t s);
// batched affine conversions (Montgomery's simultaneous inversion, k_inv.hip): r_i pk_i -> pk_aff, H(m) -> h_aff
void launch_batch_inv(const uint32_t* src, uint32_t src_stride, int w0, uint32_t* dst, uint32_t n, hipStream_t s);
void launch_pk_affine(const PipelineBuffers& b, uint32_t n_sets, hipStream_t s);
void launch_h_affine(const PipelineBuffers& b, hipStream_t s);
// r_i sig_i -> b.rsig for the sets list[0 .. n) (all sets when list is null), G2 window tables in b.scal_tab
void launch_sig_scale(const PipelineBuffers& b, uint32_t n_sets, hipStream_t s, const uint32_t* list = nullptr);
// S_r = sum r_i sig_i over the included sets of each range, as a bucket MSM (k_msm.hip, msm.hpp).  Range r is the
// slices [range_slices[r], range_slices[r+1]); slice s is the sets [slices[2s], slices[2s+1]) (<= MSM_SLICE of
// them).  B: MSM_BUCKET_WORDS words per slice, W: MSM_WINDOW_WORDS per range; S: W_G2J SoA, stride n_ranges.
#ifndef MSM_SLICE
#define MSM_SLICE 256
#endif
#define MSM_BUCKET_WORDS (128 * W_G2J)
#define MSM_WINDOW_WORDS (16 * W_G2J)
// lane_tail: the Horner passes on two lanes per range instead of cooperative 16-lane groups (merged runs)
// tree_slices: the most slices of any range; > 2 sums each range's slices by a pairwise tree of launches before the
// window pass (latency-bound runs with short slices), else the window lanes sum them serially
void launch_sig_msm(const PipelineBuffers& b, const uint32_t* slices, uint32_t n_slices, const uint32_t* range_slices,
                    uint32_t n_ranges, uint32_t* B, uint32_t* W, uint32_t* S, hipStream_t s, bool lane_tail = false,
                    uint32_t tree_slices = 0);
// per-job error status and the per-set include mask of the batch equation
void launch_job_mask(const PipelineBuffers& b, hipStream_t s);
// P_u = sum over the unit's included sets of r_i pk_i (affine)
void launch_unit_aggregate(const PipelineBuffers& b, hipStream_t s);
// Miller lines of every unique message
void launch_miller_lines(const PipelineBuffers& b, hipStream_t s);
// the same on two lanes per message (k_miller_lines2: mid-size runs, latency)
void launch_miller_lines2(const PipelineBuffers& b, hipStream_t s);
// Miller values of the chunks (items are units when `units`, else sets): f_chunk[c] = prod over the chunk's
// active items of MillerLoop(P_item, H(m_item)), one lane per chunk, the Fp12 squarings shared
void launch_miller_accx(const PipelineBuffers& b, bool units, hipStream_t s);
void launch_miller_acc(const PipelineBuffers& b, bool units, hipStream_t s);
// the same for chunks of ONE item each, two lanes per pairing (k_miller.hip k_miller_acc2: mid-size runs, latency)
void launch_miller_acc2(const PipelineBuffers& b, bool units, hipStream_t s);
// the same on SIX lanes per chunk, one w-basis Fp2 coefficient of f per lane (k_miller_acc6: 2k-16k-pairing runs)
void launch_miller_acc6(const PipelineBuffers& b, bool units, hipStream_t s);
// the same for chunks of ONE item each, as one cooperative 128-lane workgroup per pairing (lines on the fly; small
// runs, for latency)
// (exclusive: each workgroup takes a CU to itself -- k_common.hpp exclusive_cu_lds -- for latency-bound small runs;
// BLSGPU_EXCLUSIVE_SMALL=0 turns it off everywhere)
#ifndef BLSGPU_EXCLUSIVE_SMALL
#define BLSGPU_EXCLUSIVE_SMALL 1
#endif
void launch_miller_coop(const PipelineBuffers& b, bool units, hipStream_t s, bool exclusive = false);
// Batch groups: group g covers Miller chunks [f_ranges[2g], f_ranges[2g+1]).
// reduce: F_g = prod f_chunk over chunks [f_ranges[2g], f_ranges[2g+1]) (W_FP12 SoA, stride n_groups); S_g comes
// from launch_sig_msm (or, in the fallback, from per-set scalings summed by launch_group_reduce_lane)
void launch_group_reduce(const PipelineBuffers& b, const uint32_t* f_ranges, uint32_t n_groups, uint32_t* F,
                         hipStream_t s);
// the same F_g as a product tree (k_group.hip): runs[0 .. n_runs) (first, end) chunk runs multiplied lane-serially
// into their first chunk, then the pair levels (pairs up to level_end[0], then up to level_end[1], ...: f[dst] *=
// f[src], one cooperative workgroup per pair), then F_g = f[first chunk of g]
void launch_group_tree(const PipelineBuffers& b, const uint32_t* f_ranges, uint32_t n_groups, const uint32_t* runs,
                       uint32_t n_runs, const uint32_t* pairs, const std::vector<uint32_t>& level_end, uint32_t* F,
                       hipStream_t s);
// check: ok_g = FinalExp(F_g * MillerLoop(-g1, S_g)) == 1
// (sel: check only the entries sel[0 .. n_sel), verdict q -> ok[q])
// (G: MillerLoop(-g1, S_g) precomputed by launch_group_sig_miller, W_FP12 SoA stride n_groups; null = computed here)
// (lane: one lane per check instead of a cooperative workgroup -- the fallback's large launches under load; G null)
void launch_group_check(const uint32_t* S, const uint32_t* F, uint32_t n_groups, uint8_t* ok, hipStream_t s,
                        const uint32_t* sel = nullptr, uint32_t n_sel = 0, const uint32_t* G = nullptr,
                        bool exclusive = false, bool lane = false);
// six lanes per check (k_group_check6, gt6.hpp): ok = FinalExp(F * G) == 1 with G = MillerLoop(-g1, S) precomputed
// (launch_group_sig_miller; sel: check only entries sel[0 .. n_sel), verdict q -> ok[q])
void launch_group_check6(const uint32_t* F, const uint32_t* G, uint32_t n_groups, uint8_t* ok, hipStream_t s,
                         const uint32_t* sel = nullptr, uint32_t n_sel = 0);
// the whole check on six lanes: S's Miller lines one lane per entry (k_check_lines, into `lines`: n_groups x 68 x W_LINE
// words; flags: n_groups bytes), then MillerLoop(-g1, S), F * G and the final exponentiation on six lanes per check
void launch_check6_miller(const uint32_t* S, const uint32_t* F, uint32_t n_groups, uint8_t* ok, hipStream_t s,
                          const uint32_t* sel, uint32_t n_sel, uint32_t* lines, uint8_t* flags);
// G[sel[q]] = MillerLoop(-g1, S[sel[q]]) on one lane per entry (all n_groups entries when sel is null)
void launch_group_sig_miller_sel(const uint32_t* S, uint32_t n_groups, const uint32_t* sel, uint32_t n_sel, uint32_t* G,
                                 hipStream_t s);
// lane: one lane per group (pairing.hpp miller_loop) instead of a three-wave cooperative workgroup (merged runs)
void launch_group_sig_miller(const uint32_t* S, uint32_t n_groups, uint32_t* G, hipStream_t s, bool exclusive = false,
                             bool lane = false);
// lane-per-item forms (one lane per range / sub-group) for the fallback's many tiny ranges
void launch_copy_words(uint32_t* dst, const uint32_t* src, size_t n, hipStream_t s);
void launch_group_reduce_lane(const PipelineBuffers& b, const uint32_t* set_ranges, const uint32_t* f_ranges,
                              uint32_t n_groups, uint32_t* S, uint32_t* F, hipStream_t s);
void launch_range_combine_lane(const uint32_t* S_in, const uint32_t* F_in, uint32_t n_in, const uint32_t* ranges,
                               uint32_t n_out, uint32_t* S_out, uint32_t* F_out, hipStream_t s);
// fallback sub-groups: S_out[r] = sum, F_out[r] = prod of the per-job entries ranges[2r] .. ranges[2r+1]
void launch_range_combine(const uint32_t* S_in, const uint32_t* F_in, uint32_t n_in, const uint32_t* ranges,
                          uint32_t n_out, uint32_t* S_out, uint32_t* F_out, hipStream_t s);
// pubkey table upload: decode 96-byte affine encodings into table entries, per-entry status
void launch_pk_table_fill(const uint8_t* pk96, uint32_t n, uint32_t* table_dst, int8_t* status, hipStream_t s);
// serialize the per-set aggregate (pk_jac) to 96-byte uncompressed or 48-byte compressed encodings
void launch_pk_serialize(const PipelineBuffers& b, uint32_t n_sets, uint8_t* out, uint32_t out_len, hipStream_t s);
// KeyValidate of untrusted 48/96-byte pubkeys (decode + G1 subgroup check) -> 96-byte uncompressed
void launch_key_validate(const uint8_t* pks, uint32_t n, uint32_t pk_len, uint32_t stride, uint8_t* out96,
                         int8_t* status, hipStream_t s);
// SSZ signing roots (SigningData / AttestationData hash_tree_root)
void launch_signing_roots(int kind, const uint8_t* in, uint32_t n, uint32_t in_stride, const uint8_t* domain,
                          uint32_t domain_stride, uint8_t* out, hipStream_t s);
// debug ops (blsgpu_debug_op)
void launch_debug_op(int op, uint32_t n, const uint8_t* in, uint32_t in_stride, uint8_t* out, uint32_t out_stride,
                     int32_t* status, hipStream_t s);

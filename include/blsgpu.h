/* blsgpu.h -- C ABI of the MI355X BLS12-381 signature-set verifier (libblsgpu.so).
 *
 * Drop-in boundary for Lodestar's IBlsVerifier path.  The entry points replace, one for one, what the
 * reference reaches through @chainsafe/bls / @chainsafe/blst from its worker pool:
 *
 *   blsgpu_verify / blsgpu_submit  <- BlsMultiThreadWorkerPool.verifySignatureSets
 *                                      (reference packages/beacon-node/src/chain/bls/multithread/index.ts:134-174)
 *                                      + worker verifyManySignatureSets (multithread/worker.ts:32-108)
 *                                      + verifySignatureSetsMaybeBatch (chain/bls/maybeBatch.ts:16-39)
 *   pk_bytes / set_pk_first+pk_index <- getAggregatedPubkey(set).toBytes(uncompressed) (multithread/index.ts:160,
 *                                      chain/bls/utils.ts:5-16); table mode aggregates on the GPU instead
 *   blsgpu_pubkeys_upload           <- the pubkey cache the sets draw from (state-transition
 *                                      src/cache/pubkeyCache.ts:56-77, epochContext.ts:702-705)
 *   blsgpu_destroy                  <- IBlsVerifier.close (chain/bls/interface.ts:45)
 *   blsgpu_aggregate_pubkeys        <- PublicKey.aggregate(pks).toBytes() (chain/bls/utils.ts:5-16,
 *                                      multithread/index.ts:160)
 *   blsgpu_key_validate             <- PublicKey.fromBytes(pk, CoordType.affine, validate = true) for untrusted
 *                                      keys (state-transition/src/block/processDeposit.ts:56-64,
 *                                      beacon-node/test/spec/general/bls.ts:33-42)
 *   blsgpu_signing_roots            <- computeSigningRoot (state-transition/src/util/signingRoot.ts:7-13)
 *   blsgpu_shard_jobs               <- the job sharding rule the runtime applies over devices (also restated
 *                                      by lodestar_amd/shard.py for one-process-per-GPU launches)
 *   blsgpu_route_call               <- which devices a call runs on (whole on the least-loaded device below
 *                                      "route_split_sets" sets, else split); the pool's worker choice
 *                                      (multithread/index.ts:386-401 prepareWork + the free-worker pick)
 *
 * Conventions: plain pointers and sizes, caller-owned buffers, every call copies its inputs before
 * returning (blsgpu_submit included), `int` status (0 = ok).  Per-job results use the blst error names
 * thrown by @chainsafe/blst: result 1 = valid, 0 = invalid (a well-formed signature that does not
 * verify), negative = -(BLSGPU_* error code) -> the JS side rejects the job's promise with
 * Error("BLST_ERROR: <name>") exactly where the reference throws.
 */
#ifndef BLSGPU_H
#define BLSGPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BLSGPU_ABI_VERSION 7

/* blsgpu_batch.job_flags bits (reference VerifySignatureOpts, chain/bls/interface.ts:3-18) */
#define BLSGPU_JOB_BATCHABLE 1u /* opts.batchable: the job may share a random-linear-combination group */
#define BLSGPU_JOB_URGENT 2u    /* opts.verifyOnMainThread ("no-delay"): the reference verifies such a job at once on
                                   the main thread, bypassing the pool queue (multithread/index.ts:138-151; used for the
                                   gossip block proposer signature, chain/validation/block.ts:146).  A call with an
                                   urgent job runs on the device's urgent lane: its own dispatcher, slot and streams
                                   (on a reserved CU partition when option "urgent_cus" > 0), never queued behind or
                                   merged with throughput calls (option "urgent_lane"; calls above "urgent_max_sets"
                                   sets go to the head of the device queue instead). */

enum blsgpu_code {
  BLSGPU_OK = 0,
  BLSGPU_BAD_ENCODING = 1,       /* BLST_BAD_ENCODING */
  BLSGPU_POINT_NOT_ON_CURVE = 2, /* BLST_POINT_NOT_ON_CURVE */
  BLSGPU_POINT_NOT_IN_GROUP = 3, /* BLST_POINT_NOT_IN_GROUP */
  BLSGPU_AGGR_TYPE_MISMATCH = 4, /* BLST_AGGR_TYPE_MISMATCH (unused on this path) */
  BLSGPU_VERIFY_FAIL = 5,        /* BLST_VERIFY_FAIL (unused on this path) */
  BLSGPU_PK_IS_INFINITY = 6,     /* BLST_PK_IS_INFINITY */
  BLSGPU_BAD_SCALAR = 7,         /* BLST_BAD_SCALAR (unused on this path) */
  BLSGPU_INVALID_SIZE = 8,       /* BLST_INVALID_SIZE: signature not 96/192 bytes (multithread.test.ts:100) */
  BLSGPU_EMPTY_AGGREGATE = 9,    /* EMPTY_AGGREGATE_ARRAY: aggregate set with pubkeys = [] */
  BLSGPU_EMPTY_SET = 10,         /* "Empty signature set" (maybeBatch.ts:29-31) */
  BLSGPU_DEVICE_ERROR = 11,      /* HIP failure: every job of the call is rejected, never `false` */
  BLSGPU_ERR_ARGS = 100,         /* call-level: malformed arguments */
  BLSGPU_ERR_NO_DEVICE = 101,    /* call-level: no usable MI355X */
  BLSGPU_ERR_CLOSED = 102,       /* call-level: context destroyed (QUEUE_ERROR_QUEUE_ABORTED) */
  BLSGPU_ERR_ENTROPY = 103       /* call-level: seed 0 and the OS gave no randomness for the batch scalars: the call
                                    is refused (every job -BLSGPU_DEVICE_ERROR), never run with guessable scalars */
};

typedef struct blsgpu_ctx blsgpu_ctx;

/* One verifySignatureSets submission: n_jobs jobs over n_sets signature sets.  Job j owns sets
 * [job_first_set[j], job_first_set[j+1]).  A job resolves true iff every one of its sets verifies;
 * jobs never affect each other's outcome (the reference's per-job isolation, worker.ts:76-98). */
typedef struct blsgpu_batch {
  uint32_t n_sets;
  uint32_t n_jobs;
  const uint32_t* job_first_set; /* [n_jobs + 1], non-decreasing, job_first_set[n_jobs] == n_sets */
  const uint8_t* job_flags;      /* [n_jobs] BLSGPU_JOB_BATCHABLE | BLSGPU_JOB_URGENT; NULL = none */
  /* Public keys, one of three modes (set_pk_first is [n_sets + 1], non-decreasing, starting at 0):
   *  bytes mode (pk_bytes, set_pk_first == NULL): pk_bytes[96 * i] = set i's pubkey, uncompressed affine
   *    (ZCash) -- what the pool sends today, getAggregatedPubkey(set).toBytes() (multithread/index.ts:160);
   *  bytes-aggregate mode (pk_bytes and set_pk_first): set i aggregates the keys pk_bytes[96 * k],
   *    k in [set_pk_first[i], set_pk_first[i+1]) -- the aggregate ISignatureSet of any PublicKey objects
   *    (pk.toBytes()), aggregated on the GPU; a set with no keys rejects with EMPTY_AGGREGATE_ARRAY;
   *  table mode (pk_bytes == NULL): set i aggregates device-table entries pk_index[set_pk_first[i] ..
   *    set_pk_first[i+1]) (blsgpu_pubkeys_upload); an index beyond the table fails the call with ERR_ARGS.
   * Keys are trusted (subgroup-checked when they entered the pubkey cache); malformed bytes reject the job
   * with BLST_BAD_ENCODING / BLST_POINT_NOT_ON_CURVE, an aggregate equal to the identity with
   * BLST_PK_IS_INFINITY. */
  const uint8_t* pk_bytes;
  const uint32_t* set_pk_first; /* [n_sets + 1] */
  const uint32_t* pk_index;
  const uint8_t* msgs;     /* [32 * n_sets] signing roots */
  const uint8_t* sigs;     /* [sig_stride * n_sets] untrusted signature bytes */
  const uint32_t* sig_len; /* [n_sets]: 96 (compressed) or 192 (uncompressed); else BLST_INVALID_SIZE */
  uint32_t sig_stride;
  uint64_t seed; /* random-linear-combination scalars (ChaCha20 keystream, one 64-bit word per set): 0 = a fresh
                  * 256-bit key from getrandom per call (production; BLSGPU_ERR_ENTROPY if unavailable), else a key
                  * derived from this seed (deterministic comparison runs only) */
} blsgpu_batch;
/* Identical signing roots within a call are hashed to G2 once, and within a batch group the sets that sign
 * the same root are paired once, against sum_i r_i pk_i (option "dedupe", default 1). */

typedef struct blsgpu_stats {
  uint32_t groups;             /* batch groups checked (one final exponentiation each) */
  uint32_t batch_retries;      /* failed groups re-checked per job (metric blsThreadPool.batchRetries) */
  uint32_t batch_sigs_success; /* sets accepted by a batch group (metric blsThreadPool.batchSigsSuccess) */
  uint32_t devices_used;
  double device_ms; /* wall time of the call from dispatch to completion */
  /* With option "profile" = 1: per-stage kernel time (HIP events on the launch stream, device 0 shard):
   * 0 sig_decode 1 hash_to_g2 2 pk_aggregate 3 pk_finish 4 sig_msm 5 miller_sets
   * 6 group_sig_miller 7 group_finish */
  double stage_ms[8];
  uint32_t unique_messages; /* distinct signing roots hashed to G2 */
  uint32_t pairing_units;   /* Miller loops of the batch pass (sets, or same-message units) */
  uint32_t miller_chunks;   /* Miller accumulators of the batch pass (miller_k pairings share squarings) */
  uint32_t run_sets;        /* sets of the pipeline run that stage_ms timed: a runtime slot that merged queued
                               calls into one run reports it (and stage_ms) on the first call, 0 on the others */
  uint32_t run_calls;       /* calls served by the pipeline run of this call's (first) shard: 1 = ran alone, k > 1 =
                               merged with k - 1 other queued calls (set on every call of the run) */
  uint32_t fallback_jobs;   /* clean jobs of failed groups re-checked on their own (the run's, like run_sets) */
  uint32_t fallback_miller; /* Miller loops the fallback recomputed: 0 when it reused the batch pass's per-set values
                               (per-set pairings, no same-message units) */
  uint32_t urgent_lane;     /* 1 = the call ran on a device's urgent lane (BLSGPU_JOB_URGENT) */
  double host_ms;           /* host time of the run (like run_sets): from the slot taking it (merging, packing, job
                               structure, dedupe) to its input copy being queued; the largest over the call's shards */
} blsgpu_stats;

/* Create a context on the given HIP devices (NULL / n <= 0: every visible device).  Each device runs
 * "slots" runtime slots (a slot = its HIP streams + staging, served by one long-lived dispatcher thread);
 * concurrent calls run on different slots.  Slots are created by the first call, so a "slots" value set right
 * after init is the count the device runs; later changes add or retire slots.  The library never touches the
 * environment: HIP maps the slots' streams onto GPU_MAX_HW_QUEUES hardware queues (HIP's default 4), and the
 * default slot count is chosen so the streams fit the queues the process has (blsgpu_get_option "hw_queues"). */
int blsgpu_init(const int* devices, int n_devices, blsgpu_ctx** out);
/* Waits for in-flight submissions, fails queued ones with BLSGPU_ERR_CLOSED, frees everything. */
void blsgpu_destroy(blsgpu_ctx* ctx);
int blsgpu_device_count(const blsgpu_ctx* ctx);

/* Trusted pubkey table (replicated on every device): entries [first_index, first_index + n) from
 * 96-byte uncompressed affine encodings.  Returns BLSGPU_BAD_ENCODING / _POINT_NOT_ON_CURVE for a
 * malformed entry (nothing is written in that case), BLSGPU_ERR_ARGS when first_index is beyond the current
 * table size (no gaps).  The devices decode and store their replicas concurrently (one host thread each); each
 * device's table grows under its own lock, so a call that uses the new indices before the upload returns may fail
 * with BLSGPU_ERR_ARGS on a device not yet updated, never verify against stale keys. */
int blsgpu_pubkeys_upload(blsgpu_ctx* ctx, uint32_t first_index, const uint8_t* pk96, uint32_t n);
uint32_t blsgpu_pubkeys_count(const blsgpu_ctx* ctx);

/* Synchronous verification.  job_result[n_jobs]: 1 valid / 0 invalid / -code.  Returns a call-level
 * status (BLSGPU_OK even when some jobs are invalid or rejected; a HIP failure rejects the jobs of the
 * affected shard with -BLSGPU_DEVICE_ERROR). */
int blsgpu_verify(blsgpu_ctx* ctx, const blsgpu_batch* batch, int8_t* job_result, blsgpu_stats* stats);

/* Asynchronous verification: inputs are copied before return; `done(user, status)` runs on a runtime
 * dispatcher thread once job_result / stats are written (status BLSGPU_ERR_CLOSED when the context was
 * destroyed before the call ran).  For the N-API addon's threadsafe-function bridge. */
typedef void (*blsgpu_done_cb)(void* user, int status);
int blsgpu_submit(blsgpu_ctx* ctx, const blsgpu_batch* batch, int8_t* job_result, blsgpu_stats* stats,
                  blsgpu_done_cb done, void* user);

/* Tunables ("slots" may not be changed from a done callback: BLSGPU_ERR_ARGS): "group_sets" (sets per batch group before a new one opens, default 1024), "group_adapt"
 * (while a device sees invalid sets, its batch groups shrink to the size that minimises the expected work of a group's
 * final exponentiation against re-checking a failed group's clean jobs -- 32 sets at 1% invalid, group_sets when all
 * are valid; 0/1, default 1.  Until the runtime stopped returning outgrown slot buffers to the stream-ordered pool
 * during operation, fresh processes verifying C5-like calls with it answered false for valid jobs in ~6% of runs),
 * "slots" (runtime slots
 * per device, 1..64; default by hardware queues), "max_devices" (devices one call may shard over, default all),
 * "dedupe" (message dedupe + same-message pairing, 0/1, default 1), "miller_k" (pairings per Miller
 * accumulator sharing its Fp12 squarings, 1..64; default 0 = by run size: 1 below 131072 pairings, 2 below
 * 262144, else 4), "merge_sets" (a runtime slot merges calls
 * already queued on its device into one pipeline run of up to this many sets -- jobs and results stay per
 * call -- default 131072, 0 = never), "pipeline_depth" (runs a device keeps in flight, default 3: consecutive runs
 * alternate between the device's two stream pairs, so two runs' message chains overlap and a third run's decode /
 * pubkey work fills the gaps; a deeper pipeline only queues), "merge_wait_us" (while runs are in
 * flight, a slot forming a run waits up to this long for more calls to merge, default 2000; an idle device starts
 * at once), "idle_wait_us" (an idle device lingers up to this long while calls keep arriving, default 0), "merge_balance"
 * (a backlog above merge_sets is cut into equal runs, 0/1, default 0), "miller_lanes" (lanes per Miller accumulation chunk: 0 = auto, the default -- two lanes
 * for one-item chunks (each holding half of f), one lane for shared-squaring chunks; 1 = one lane; 2 = two lanes; 3 =
 * lane pairs; 6 = six lanes),
 * "lines_lanes" (lanes per message of the Miller lines: 1, or 2 = lane pairs (default)), "msm_slice_mid" (MSM slice length of runs
 * of 1k-32k sets, 8..256, default 32), "msm_tree" (those runs sum each range's slices by a pairwise tree, 0/1,
 * default 1), "f_run_max" (merged runs: longest lane-serial run of the F product tree, a power of two, default 16),
 * "coop_max" / "coop_g2_max" (runs of <= this many pairings / sets take the cooperative Miller loops / [|z|] chains,
 * default 512 / 4096), "coop_excl_max" (cooperative workgroups take a CU each in runs of <= this many items, default
 * 512), "rsig_spec" (small idle runs form every r_i sig_i beside the batch pass for a possible fallback, 0/1, default
 * 1), "spec_large" (runs above small_max that find the device idle start their MSM speculatively after the decode, as
 * small ones do, 0/1, default 1), "spec_gsm" (such a speculative run's MillerLoop(-g1, S) follows its MSM on the other
 * stream pair's message stream instead of the run's signature stream, 0/1, default 0: measured equal), "fb_lane_min"
 * (fallback check launches of >= this many checks in large runs take one lane per check, default
 * 256, 0 = never), "route_split_sets" (see blsgpu_route_call, default 16384), "acc6_max" (runs of one-item Miller chunks up to this many
 * take the six-lane accumulation, default 16384; "miller_lanes" 6 forces it), "miller_pairs" (larger runs take the
 * lane-pair accumulation, every Fp2 split over two lanes at two waves per SIMD, 0/1, default 0; "miller_lanes" 3
 * forces it for every run), "small_max" (runs of <= this many sets are latency-first: on an idle device the
 * parallel pubkey branch and r_i sig_i, cooperative fallback checks; default 4096), "fb_direct_min" (large runs under
 * load with >= this many retried jobs check each one directly, default 1024, 0 = never), "fb_check6" (those checks: 0
 * one lane each, 1 Miller loop on one lane and the final exponentiation on six, 2 both on six lanes; default 2),
 * "fb_force_busy" (tests: every run's fallback takes the under-load forms, 0/1, default 0), "keep_f" (the fallback reuses
 * the batch pass's per-set Miller values instead of re-running the loops, 0/1, default 1), "keep_copy" (how they are
 * copied aside: 0 hipMemcpyAsync, 1 a copy kernel; default 0), "early_release" /
 * "tail_on_msg" / "copy_stream" (run-formation experiments, 0/1, default 0: a run leaves the pipeline count when its
 * message branch is done / the group stage on the pair's high-priority message stream / the input copy on the table
 * stream),
 * "urgent_lane" (calls with a BLSGPU_JOB_URGENT job run on the device's urgent lane, 0/1, default 1), "urgent_max_sets"
 * (larger urgent calls are queued at the head of the device queue instead, default 512), "urgent_excl" (urgent runs
 * may use the exclusive-CU padding of the cooperative kernels, 0/1, default 0), "urgent_wait_us" (the urgent dispatcher
 * lingers this long after an urgent call for more of a burst, merged into one run, default 300), "urgent_cus" (CUs per device reserved
 * for the urgent lane's streams, a multiple of 8 up to 128, 0 = no partition: the lane's streams take the highest
 * priority; CU mask bits [0, urgent_cus), which the driver deals round-robin over the XCDs) and "urgent_isolate" (with a
 * partition, the pipeline streams are masked off it; 2: and the urgent streams are left unmasked at the highest
 * priority, so an idle chip is theirs too; 3, diagnostics: the pipeline streams masked with every CU; 0..3) -- these two only before the first call (the
 * streams are created with it; BLSGPU_ERR_ARGS afterwards), "blocking_sync" (the dispatcher threads block on their
 * runs' completion events instead of spinning, 0/1, default 1; before the first call only), "pipeline_prio" (the
 * pipeline's message and tail streams take the device's highest priority, 0/1, default 1; before the first call only),
 * "lane_tail_min" / "lane_tail_parts" (runs of >= lane_tail_min sets take lane forms of the Horner passes (bit 0)
 * and of MillerLoop(-g1, S) (bit 1) instead of the cooperative workgroups; default 0 = never, parts 3), "serial"
 * (diagnostics: every branch of a run on one stream, so each kernel runs alone on the chip; 0/1, default 0), "profile" (per-stage kernel times in
 * blsgpu_stats.stage_ms, 0/1), "group_policy" (0 = batch groups of >= group_sets sets, the default; 1 = the
 * reference pool's grouping: calls split into <= 128-set jobs (chunkifyMaximizeChunkSize(sets, 128),
 * multithread/index.ts:156), packed into >= 128-set worker requests (prepareWork, index.ts:386-401), each
 * request's batchable jobs checked in chunks of >= 16 jobs (worker.ts:17,56), so batch_retries and
 * batch_sigs_success count the reference's units).  Applies to calls submitted afterwards. */
int blsgpu_set_option(blsgpu_ctx* ctx, const char* key, int64_t value);
/* Current value of a tunable (the keys of blsgpu_set_option; "slots" = the slots device 0 runs, or will create
 * on the first call) or of a read-only property: "hw_queues" (the GPU_MAX_HW_QUEUES HIP runs with),
 * "abi_version", "spurious_groups" (batch groups whose equation failed although every job of theirs verified on its
 * own in the fallback, over the context's life: zero unless a kernel computed a group's equation wrong; each is also
 * logged to stderr). */
int blsgpu_get_option(const blsgpu_ctx* ctx, const char* key, int64_t* value);

/* chunkifyMaximizeChunkSize(arr of len items, min_per_chunk) (multithread/utils.ts:4-19): writes the first
 * index of every chunk and len to chunk_first[0 .. *n_chunks] (room for len / min_per_chunk + 2 entries).
 * Pure host code; the rule group_policy 1 applies. */
int blsgpu_chunkify(uint32_t len, uint32_t min_per_chunk, uint32_t* chunk_first, uint32_t* n_chunks);

/* PublicKey.aggregate(set pubkeys).toBytes() for every set of `b` (only n_sets and the pubkey fields are
 * read; any of the three modes): out[out_len * i], out_len 96 (uncompressed) or 48 (compressed);
 * status[i] = 0, EMPTY_AGGREGATE (no keys) or the first malformed key's code.  An aggregate equal to the
 * identity is encoded as the identity. */
int blsgpu_aggregate_pubkeys(blsgpu_ctx* ctx, const blsgpu_batch* b, uint8_t* out, uint32_t out_len,
                             int8_t* status);

/* KeyValidate of n untrusted pubkeys (pks[stride * i], pk_len 48 compressed or 96 uncompressed): status[i]
 * = 0 or BAD_ENCODING / POINT_NOT_ON_CURVE / PK_IS_INFINITY / POINT_NOT_IN_GROUP; out96 (nullable)
 * receives the uncompressed encoding of every valid key (bytes-mode input of blsgpu_verify). */
int blsgpu_key_validate(blsgpu_ctx* ctx, uint32_t n, const uint8_t* pks, uint32_t pk_len, uint32_t stride,
                        uint8_t* out96, int8_t* status);

/* Signing roots: out32[32 i] = hash_tree_root(SigningData{object_root_i, domain_i}) where object_root_i is
 * objects[object_stride * i] itself (BLSGPU_ROOT_OBJECT, 32 B) or hash_tree_root of the SSZ-serialized
 * AttestationData there (BLSGPU_ROOT_ATTESTATION_DATA, 128 B); domain_i = domains[domain_stride * i]
 * (domain_stride 0: one domain for all). */
#define BLSGPU_ROOT_OBJECT 0
#define BLSGPU_ROOT_ATTESTATION_DATA 1
int blsgpu_signing_roots(blsgpu_ctx* ctx, int kind, uint32_t n, const uint8_t* objects, uint32_t object_stride,
                         const uint8_t* domains, uint32_t domain_stride, uint8_t* out32);

/* The runtime's job sharding: part k = jobs [part_first_job[k], part_first_job[k+1]) of n_parts contiguous,
 * cost-balanced parts (cost = sets + aggregated pubkeys / 256; set_pk_first nullable).  Pure host code. */
int blsgpu_shard_jobs(const uint32_t* job_first_set, const uint32_t* set_pk_first, uint32_t n_jobs,
                      uint32_t n_parts, uint32_t* part_first_job);

/* The runtime's call routing: a call of n_sets sets goes to k = min(n_devices, max(1, n_sets / split_sets)) devices
 * (option "route_split_sets", default 16384: a gossip call runs whole on one device, an epoch-scale call splits), the
 * k least loaded by device_load[] (cost of their queued and running shards), ties broken by distance from `start`;
 * out_devices[0 .. k) in shard order (ascending), *n_out = k.  Pure host code (lodestar_amd/shard.py route_call
 * restates it). */
int blsgpu_route_call(uint32_t n_sets, uint32_t n_devices, const int64_t* device_load, int64_t split_sets,
                      uint32_t start, uint32_t* out_devices, uint32_t* n_out);

/* The batch scalar words blsgpu_verify would use for `b` (only n_sets, n_jobs, job_first_set, job_flags and seed
 * are read): words[i] for set i, 0 = r = 1 (a single-set non-batchable job: CoreVerify).  With seed 0 every call
 * draws a fresh key, so two calls differ.  Returns BLSGPU_ERR_ENTROPY when seed is 0 and the OS gives no
 * randomness.  Pure host code. */
int blsgpu_batch_scalars(const blsgpu_batch* b, uint64_t* words);

/* Test hook: fault injection, process-wide, available only when the process was started with the environment
 * variable BLSGPU_FAULT_INJECTION=1 (read once; otherwise every call returns BLSGPU_ERR_ARGS and nothing is armed).
 * After `skip` more events, the next `count` events fail:
 *   BLSGPU_INJECT_ENTROPY: an entropy draw (seed-0 calls, blsgpu_batch_scalars) -> BLSGPU_ERR_ENTROPY;
 *   BLSGPU_INJECT_DEVICE: a pipeline run, once its batch pass completed, as if a HIP call had failed -> every job
 *     of every call in that run -BLSGPU_DEVICE_ERROR (never 0); the dispatcher keeps serving later calls.
 * count 0 disarms. */
#define BLSGPU_INJECT_ENTROPY 1
#define BLSGPU_INJECT_DEVICE 2
int blsgpu_debug_inject(int what, int64_t skip, int64_t count);

/* "BLST_INVALID_SIZE", ... for job codes; NULL for unknown codes. */
const char* blsgpu_code_name(int code);

/* Test hook: run one pipeline stage element-wise on device 0 (canonical big-endian encodings).
 * op: 0 fp_mul(48,48->48) 1 sig_decode(192+len -> status,192) 2 hash_to_g2(32->192)
 *     3 miller(96,192->576) 4 final_exp(576->576) 5 g1_mul_u64(96,8->96) 6 g2_mul_u64(192,8->192)
 *     7 sign(sk32||msg32 -> 96 compressed) 8 sk_to_pk(sk32 -> 96 uncompressed)   (workload generation)
 *     9 g2_mul_scalar_word(192,8 -> 192; out_stride >= 2880) 10 g1_mul_scalar_word(96,8 -> 96; >= 1440):
 *       the batch scalar r = a + b*lambda of a scalar word w (a = 2 lo + 1 - 2^32, b = 2 hi + 1 - 2^32 from w's
 *       32-bit halves, lambda = -z^2), word 0 = r = 1
 *     11 fp_lc(raw limbs: 15 x 14 LE words -> 14 words): the lazily reduced combination x0 + .. + x6 - x7 - .. - x14
 *     16 final_exp / 17 miller (the cooperative GT engine, 576 / 288 -> 576)
 *     18 lane-pair G2 arithmetic (fp2x.hpp) against the one-lane forms: P, Q affine (384) -> [|z|]P affine (192);
 *        status = bitmask of the cases (add, add doubling / infinity branches, dbl, mixed add, psi, psi^2, [|z|],
 *        Fp2 product / square) where the lane-pair result differs
 * Strides below an op's element size, and unknown ops, are refused with BLSGPU_ERR_ARGS.
 * Returns BLSGPU_OK or an error. */
int blsgpu_debug_op(blsgpu_ctx* ctx, int op, uint32_t n, const uint8_t* in, uint32_t in_stride,
                    uint8_t* out, uint32_t out_stride, int32_t* status);

#ifdef __cplusplus
}
#endif
#endif /* BLSGPU_H */

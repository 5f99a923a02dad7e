"use strict";
/**
 * BlsGpuVerifier: the IBlsVerifier drop-in (reference packages/beacon-node/src/chain/bls/interface.ts:20-46)
 * over the blsgpu N-API addon.  It replaces BlsMultiThreadWorkerPool (multithread/index.ts) with the same
 * observable behaviour:
 *
 *   - verifySignatureSets(sets, opts) -> Promise<boolean>: true iff every set is valid; false if a
 *     well-formed set fails the pairing equation; rejects with "BLST_ERROR: <CODE>" when a signature
 *     fails to deserialize (maybeBatch.ts:23,36 -> Signature.fromBytes throws; multithread.test.ts:93-100),
 *     with "EMPTY_AGGREGATE_ARRAY" for an aggregate without pubkeys (utils.ts:11), and with the device
 *     status for a device error (never `false`, index.ts:368-375).
 *   - batchable jobs are buffered for up to MAX_BUFFER_WAIT_MS or until more than MAX_BUFFERED_SIGS sets
 *     are waiting, then submitted together; every job keeps its own result (index.ts:41-57, 238-285).
 *     Non-batchable jobs are submitted on the next macrotask, so a synchronous loop of calls coalesces
 *     into one submission (index.ts:276-283).
 *   - close() rejects buffered and queued jobs with QUEUE_ERROR_QUEUE_ABORTED (index.ts:176-197) and
 *     destroys the device context.
 *
 * Pubkeys.  A set's pubkey (single) or each of its pubkeys (aggregate) is one of:
 *   - a validator index (number) into the device table filled by uploadPubkeys() from index2pubkey
 *     (state-transition/src/cache/pubkeyCache.ts:56-77) -- GPU aggregation, no main-thread
 *     PublicKey.aggregate (utils.ts:5-16);
 *   - an object registered with registerPubkey(obj, index) (a blst PublicKey, mapped by identity);
 *   - any PublicKey-like object with toBytes() (96 uncompressed affine bytes, PointFormat.uncompressed),
 *     or those 96 bytes as a Uint8Array -- what the pool sends its workers today (index.ts:160).  Aggregate
 *     sets of such keys (the gossip attestation call, attestation.ts:131-138) are aggregated on the GPU
 *     from the per-key bytes (bytes-aggregate mode), so no caller needs a registration pass.
 * A job is in table mode when all its keys are indexed, in bytes mode otherwise; a flush that mixes both
 * is split into one submission per mode.
 *
 * Metrics: the pool's blsThreadPool.* / bls.* series (metrics/metrics/lodestar.ts:382-458) are fed with the
 * GPU as the worker (workerId = "gpu"): jobsWorkerTime, timePerSigSet, jobWaitTime, queueLength,
 * totalJobsGroupsStarted, totalJobsStarted, totalSigSetsStarted, latencyToWorker, latencyFromWorker,
 * successJobsSignatureSetsCount, errorJobsSignatureSetsCount, batchRetries, batchSigsSuccess,
 * mainThreadDurationInThreadPool, aggregatedPubkeys.
 *
 * Also exported: BlsGpuSingleThreadVerifier (chain/bls/singleThread.ts:7-40 semantics: every call verified
 * on its own, immediately, with the maybe-batch rule), verifySignatureSet (state-transition
 * signatureSets.ts:24-38: Signature.verify / verifyAggregate), and the spec-conformance entry points
 * fastAggregateVerify / ethFastAggregateVerify (beacon-node/test/spec/general/bls.ts: untrusted keys
 * through KeyValidate, any error -> false).
 */
const path = require("path");

// CommonJS implementation (.cjs, so it stays CommonJS inside the "type": "module" beacon-node package); ESM callers
// import it through index.js, TypeScript through index.d.ts.  The module never writes process.env: the runtime sizes
// its slots to the hardware queues HIP gives the process (include/blsgpu.h blsgpu_init).
const addon = require(path.join(__dirname, "blsgpu_napi.node"));

const MAX_BUFFERED_SIGS = 32; // multithread/index.ts:48
const MAX_BUFFER_WAIT_MS = 100; // multithread/index.ts:57
const QUEUE_ABORTED = "QUEUE_ERROR_QUEUE_ABORTED"; // util/queue/errors.ts QueueErrorCode.QUEUE_ABORTED
const SIG_STRIDE = 192;

// job flags (include/blsgpu.h BLSGPU_JOB_*)
const JOB_BATCHABLE = 1;
const JOB_URGENT = 2;

// job codes (include/blsgpu.h enum blsgpu_code)
const CODE_EMPTY_AGGREGATE = 9;
const CODE_EMPTY_SET = 10;

class QueueError extends Error {
  constructor(type) {
    super(type.code);
    this.type = type;
  }
}

const SignatureSetType = {single: "single", aggregate: "aggregate"}; // signatureSets.ts:5-8

function jobError(code) {
  const name = addon.codeName(code) || `BLSGPU_${code}`;
  if (code === CODE_EMPTY_SET || code === CODE_EMPTY_AGGREGATE) return new Error(name);
  return new Error(`BLST_ERROR: ${name}`);
}

class BlsGpuVerifier {
  /**
   * @param {{devices?: number[], groupSets?: number, groupPolicy?: number, seed?: number}} opts
   * @param {{metrics?: object, logger?: object}} modules
   */
  constructor(opts = {}, modules = {}) {
    this.ctx = addon.init(opts.devices || null);
    if (opts.groupSets) addon.setOption(this.ctx, "group_sets", opts.groupSets);
    // 1 = the pool's job / request / chunk structure (batchRetries / batchSigsSuccess in the reference's units)
    if (opts.groupPolicy) addon.setOption(this.ctx, "group_policy", opts.groupPolicy);
    this.seed = opts.seed || 0; // 0 = OS CSPRNG batch scalars; fixed only for comparison runs
    // verifyOnMainThread calls are latency-critical exceptions to the pool (the block proposer signature): they run on
    // the device's urgent lane.  The single-thread verifier sends every call that way and keeps the shared pipeline.
    this.urgentMainThread = true;
    this.metrics = modules.metrics || null;
    this.closed = false;
    this.bufferedJobs = null; // {jobs, sigCount, timeout}
    this.queued = []; // non-batchable jobs waiting for the next macrotask
    this.queuedTimer = null;
    this.inflight = new Set();
    this.pkIndexOf = new WeakMap();
    this.stats = {submissions: 0, jobs: 0, sets: 0, groups: 0, batchRetries: 0, batchSigsSuccess: 0, uniqueMessages: 0};
    this.queueLength = 0; // submissions on the device (blsThreadPool.queueLength)
    const m = this.metrics && this.metrics.blsThreadPool;
    if (m && m.queueLength && m.queueLength.addCollect) m.queueLength.addCollect(() => m.queueLength.set(this.queueLength));
  }

  /** index2pubkey sync: entries [firstIndex, firstIndex + n) as 96-byte uncompressed affine encodings. */
  uploadPubkeys(firstIndex, pk96) {
    addon.uploadPubkeys(this.ctx, firstIndex, pk96);
  }

  registerPubkey(obj, index) {
    this.pkIndexOf.set(obj, index);
  }

  get deviceCount() {
    return addon.deviceCount(this.ctx);
  }

  /** A runtime tunable or property (include/blsgpu.h blsgpu_get_option: "slots", "hw_queues", "group_sets", ...). */
  getOption(key) {
    return addon.getOption(this.ctx, key);
  }

  /**
   * IBlsVerifier.verifySignatureSets (interface.ts:20-43).
   * @param {Array<{type: string, pubkey?: any, pubkeys?: any[], signingRoot: Uint8Array, signature: Uint8Array}>} sets
   * @param {{batchable?: boolean, verifyOnMainThread?: boolean}} opts
   * @returns {Promise<boolean>}
   */
  async verifySignatureSets(sets, opts = {}) {
    if (this.closed) throw new QueueError({code: QUEUE_ABORTED});
    if (this.metrics && this.metrics.bls && this.metrics.bls.aggregatedPubkeys) {
      let n = 0;
      for (const s of sets) if (s.type === SignatureSetType.aggregate) n += s.pubkeys.length;
      this.metrics.bls.aggregatedPubkeys.inc(n);
    }
    // the pool path chunks the call into jobs and ANDs their results: no jobs -> "Empty results array"
    // (multithread/index.ts:169-171); the main-thread path throws "Empty signature set" (maybeBatch.ts:29-31)
    if (sets.length === 0) throw new Error(opts.verifyOnMainThread ? "Empty signature set" : "Empty results array");
    const job = this.encodeJob(sets, opts);
    job.addedTimeMs = Date.now();
    const code = await new Promise((resolve, reject) => {
      job.resolve = resolve;
      job.reject = reject;
      if (opts.batchable && !opts.verifyOnMainThread) {
        if (!this.bufferedJobs) {
          this.bufferedJobs = {jobs: [], sigCount: 0, timeout: setTimeout(() => this.flushBuffered(), MAX_BUFFER_WAIT_MS)};
        }
        this.bufferedJobs.jobs.push(job);
        this.bufferedJobs.sigCount += job.sets.length;
        if (this.bufferedJobs.sigCount > MAX_BUFFERED_SIGS) {
          clearTimeout(this.bufferedJobs.timeout);
          this.flushBuffered();
        }
      } else if (opts.verifyOnMainThread) {
        // latency-critical (block proposal, interface.ts:8-17): no buffering at all, and on the device the urgent
        // lane (BLSGPU_JOB_URGENT)
        job.mainThread = true;
        this.dispatch([job]);
      } else {
        this.queued.push(job);
        if (!this.queuedTimer) {
          this.queuedTimer = setTimeout(() => {
            this.queuedTimer = null;
            const jobs = this.queued.splice(0, this.queued.length);
            this.dispatch(jobs);
          }, 0);
        }
      }
    });
    if (code < 0) throw jobError(-code);
    return code === 1;
  }

  /** IBlsVerifier.close (interface.ts:45). */
  async close() {
    if (this.closed) return;
    this.closed = true;
    const pending = [];
    if (this.bufferedJobs) {
      clearTimeout(this.bufferedJobs.timeout);
      pending.push(...this.bufferedJobs.jobs);
      this.bufferedJobs = null;
    }
    if (this.queuedTimer) clearTimeout(this.queuedTimer);
    this.queuedTimer = null;
    pending.push(...this.queued.splice(0, this.queued.length));
    for (const job of pending) job.reject(new QueueError({code: QUEUE_ABORTED}));
    // in-flight submissions complete (the device finishes them) before the context is freed
    await Promise.allSettled(Array.from(this.inflight));
    addon.close(this.ctx);
  }

  // ------------------------------------------------------------------------------------ internals
  flushBuffered() {
    const b = this.bufferedJobs;
    this.bufferedJobs = null;
    if (b && b.jobs.length) this.dispatch(b.jobs);
  }

  pkRef(pk) {
    if (typeof pk === "number") return {index: pk};
    if (pk instanceof Uint8Array) return {bytes: pk};
    if (pk && typeof pk === "object") {
      const idx = this.pkIndexOf.get(pk);
      const ref = {};
      if (idx !== undefined) ref.index = idx;
      // keep the bytes too (when the object serializes), so a job mixing registered and plain keys can go
      // in bytes-aggregate mode
      if (typeof pk.toBytes === "function") ref.bytes = pk.toBytes();
      if (ref.index !== undefined || ref.bytes !== undefined) return ref;
    }
    throw new TypeError("BlsGpuVerifier: pubkey must be an index, a registered object, a PublicKey or 96 bytes");
  }

  encodeJob(sets, opts) {
    const enc = [];
    let allIndexed = true;
    for (const s of sets) {
      const refs = s.type === SignatureSetType.aggregate ? s.pubkeys.map((p) => this.pkRef(p)) : [this.pkRef(s.pubkey)];
      for (const r of refs) if (r.index === undefined) allIndexed = false;
      enc.push({refs, msg: s.signingRoot, sig: s.signature, aggregate: s.type === SignatureSetType.aggregate});
    }
    if (!allIndexed) {
      for (const e of enc)
        for (const r of e.refs)
          if (r.bytes === undefined || r.bytes.length !== 96)
            throw new TypeError("BlsGpuVerifier: pubkeys of a bytes-mode job must serialize to 96 uncompressed bytes");
    }
    return {sets: enc, table: allIndexed, batchable: !!opts.batchable};
  }

  dispatch(jobs) {
    const table = jobs.filter((j) => j.table);
    const bytes = jobs.filter((j) => !j.table);
    if (table.length) this.submit(table, true);
    if (bytes.length) this.submit(bytes, false);
  }

  submit(jobs, tableMode) {
    let nSets = 0;
    let nPk = 0;
    for (const j of jobs) {
      nSets += j.sets.length;
      for (const s of j.sets) nPk += s.refs.length;
    }
    const jobFirstSet = new Uint32Array(jobs.length + 1);
    const jobFlags = new Uint8Array(jobs.length);
    const msgs = new Uint8Array(32 * nSets);
    const sigs = new Uint8Array(SIG_STRIDE * nSets);
    const sigLen = new Uint32Array(nSets);
    const setPkFirst = new Uint32Array(nSets + 1);
    const req = {jobFirstSet, jobFlags, msgs, sigs, sigLen, sigStride: SIG_STRIDE, seed: this.seed, setPkFirst};
    let pkIndex, pkBytes;
    if (tableMode) {
      pkIndex = req.pkIndex = new Uint32Array(Math.max(nPk, 1));
    } else {
      pkBytes = req.pkBytes = new Uint8Array(Math.max(96 * nPk, 96));  // bytes-aggregate mode
    }
    let i = 0;
    let k = 0;
    const now = Date.now();
    const m = this.metrics && this.metrics.blsThreadPool;
    jobs.forEach((j, ji) => {
      jobFirstSet[ji] = i;
      // BLSGPU_JOB_BATCHABLE, and BLSGPU_JOB_URGENT for verifyOnMainThread jobs: the runtime runs those on the
      // device's urgent lane, never queued behind or merged with the gossip flood (multithread/index.ts:138-151)
      jobFlags[ji] = (j.batchable ? JOB_BATCHABLE : 0) | (j.mainThread && this.urgentMainThread ? JOB_URGENT : 0);
      if (m && m.jobWaitTime && j.addedTimeMs) m.jobWaitTime.observe((now - j.addedTimeMs) / 1000);
      for (const s of j.sets) {
        msgs.set(s.msg.subarray(0, 32), 32 * i);
        const sl = s.sig.length;
        sigLen[i] = sl; // 96 / 192, anything else -> BLST_INVALID_SIZE for this job
        sigs.set(s.sig.subarray(0, Math.min(sl, SIG_STRIDE)), SIG_STRIDE * i);
        setPkFirst[i] = k;
        for (const r of s.refs) {
          if (tableMode) pkIndex[k] = r.index;
          else pkBytes.set(r.bytes, 96 * k);
          k++;
        }
        i++;
      }
    });
    jobFirstSet[jobs.length] = nSets;
    setPkFirst[nSets] = k;
    if (m) {
      if (m.totalJobsGroupsStarted) m.totalJobsGroupsStarted.inc(1);
      if (m.totalJobsStarted) m.totalJobsStarted.inc(jobs.length);
      if (m.totalSigSetsStarted) m.totalSigSetsStarted.inc(nSets);
    }
    const submitNs = process.hrtime.bigint();
    this.queueLength += 1;
    const p = addon.submit(this.ctx, req).then(
      (out) => {
        this.queueLength -= 1;
        const st = this.stats;
        st.submissions++;
        st.jobs += jobs.length;
        st.sets += nSets;
        st.groups += out.groups;
        st.batchRetries += out.batchRetries;
        st.batchSigsSuccess += out.batchSigsSuccess;
        st.uniqueMessages += out.uniqueMessages;
        if (out.urgentLane) st.urgentCalls = (st.urgentCalls || 0) + 1;
        let okSets = 0;
        let errSets = 0;
        jobs.forEach((j, ji) => (out.results[ji] < 0 ? (errSets += j.sets.length) : (okSets += j.sets.length)));
        if (m) {
          // the device is the worker: its time is the call's device phase; the rest is host <-> device latency
          const totalSec = Number(process.hrtime.bigint() - submitNs) / 1e9;
          const devSec = out.deviceMs / 1000;
          if (m.jobsWorkerTime) m.jobsWorkerTime.inc({workerId: "gpu"}, devSec);
          if (m.timePerSigSet && nSets) m.timePerSigSet.observe(devSec / nSets);
          if (m.latencyToWorker) m.latencyToWorker.observe(Math.max(0, (totalSec - devSec) / 2));
          if (m.latencyFromWorker) m.latencyFromWorker.observe(Math.max(0, (totalSec - devSec) / 2));
          if (m.successJobsSignatureSetsCount) m.successJobsSignatureSetsCount.inc(okSets);
          if (m.errorJobsSignatureSetsCount) m.errorJobsSignatureSetsCount.inc(errSets);
          if (m.batchRetries) m.batchRetries.inc(out.batchRetries);
          if (m.batchSigsSuccess) m.batchSigsSuccess.inc(out.batchSigsSuccess);
          if (m.mainThreadDurationInThreadPool && jobs.some((j) => j.mainThread))
            m.mainThreadDurationInThreadPool.observe(totalSec);
        }
        jobs.forEach((j, ji) => j.resolve(out.results[ji]));
      },
      (err) => {
        this.queueLength -= 1;
        // call-level failure (device error, closed context): reject every job, never resolve false
        for (const j of jobs) j.reject(err.code === QUEUE_ABORTED ? new QueueError({code: QUEUE_ABORTED}) : err);
      }
    );
    this.inflight.add(p);
    p.finally(() => this.inflight.delete(p));
  }
}

/**
 * BlsSingleThreadVerifier semantics (chain/bls/singleThread.ts:7-40): every call is verified on its own,
 * immediately (no buffering, no batching with other calls), by verifySignatureSetsMaybeBatch over its sets;
 * errors reject.  Same device path: one non-batchable job per call.
 */
class BlsGpuSingleThreadVerifier extends BlsGpuVerifier {
  constructor(opts = {}, modules = {}) {
    super(opts, modules);
    // every call is "main thread" here, so none is an exception: calls share the device pipeline (no urgent lane, which
    // runs one burst of calls at a time)
    this.urgentMainThread = false;
  }

  async verifySignatureSets(sets) {
    if (sets.length === 0) throw new Error("Empty signature set");
    return super.verifySignatureSets(sets, {verifyOnMainThread: true});
  }
}

/**
 * verifySignatureSet (state-transition/src/util/signatureSets.ts:24-38): single -> Signature.verify,
 * aggregate -> Signature.verifyAggregate (FastAggregateVerify over trusted keys).  Rejects like
 * Signature.fromBytes(validate = true) on a malformed signature.
 */
async function verifySignatureSet(verifier, set) {
  return verifier.verifySignatureSets([set], {verifyOnMainThread: true});
}

const G1_INFINITY_48 = (() => {
  const b = new Uint8Array(48);
  b[0] = 0xc0;
  return b;
})();
const G2_INFINITY_96 = (() => {
  const b = new Uint8Array(96);
  b[0] = 0xc0;
  return b;
})();
const sameBytes = (a, b) => a.length === b.length && a.every((x, i) => x === b[i]);

/**
 * fast_aggregate_verify of the spec runner (beacon-node/test/spec/general/bls.ts): untrusted 48-byte keys
 * through KeyValidate (PublicKey.fromBytes(validate = true)), the signature through Signature.fromBytes
 * (validate = true); any error -> false.
 */
async function fastAggregateVerify(verifier, pubkeys48, message, signature) {
  if (pubkeys48.length === 0) return false; // EMPTY_AGGREGATE_ARRAY -> caught -> false
  const flat = new Uint8Array(48 * pubkeys48.length);
  pubkeys48.forEach((p, i) => flat.set(p.subarray(0, 48), 48 * i));
  if (pubkeys48.some((p) => p.length !== 48)) return false;
  const kv = addon.keyValidate(verifier.ctx, flat, 48);
  if (kv.status.some((s) => s !== 0)) return false;
  const keys = [];
  for (let i = 0; i < pubkeys48.length; i++) keys.push(kv.pk96.subarray(96 * i, 96 * i + 96));
  try {
    return await verifier.verifySignatureSets(
      [{type: SignatureSetType.aggregate, pubkeys: keys, signingRoot: message, signature}],
      {verifyOnMainThread: true}
    );
  } catch (e) {
    return false;
  }
}

/** eth_fast_aggregate_verify (spec runner): no keys + infinity signature -> true; an infinity key -> false. */
async function ethFastAggregateVerify(verifier, pubkeys48, message, signature) {
  if (pubkeys48.length === 0 && sameBytes(signature, G2_INFINITY_96)) return true;
  if (pubkeys48.some((p) => sameBytes(p, G1_INFINITY_48))) return false;
  return fastAggregateVerify(verifier, pubkeys48, message, signature);
}

module.exports = {
  BlsGpuVerifier,
  BlsGpuSingleThreadVerifier,
  verifySignatureSet,
  fastAggregateVerify,
  ethFastAggregateVerify,
  QueueError,
  SignatureSetType,
  MAX_BUFFERED_SIGS,
  MAX_BUFFER_WAIT_MS,
  JOB_BATCHABLE,
  JOB_URGENT,
  addon,
};

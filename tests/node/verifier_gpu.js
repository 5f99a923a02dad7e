"use strict";
// GPU parity of the JS drop-in (lodestar_amd/node/BlsGpuVerifier.cjs) against tests/golden/verify_sets.json,
// mirroring the reference's packages/beacon-node/test/e2e/chain/bls/multithread.test.ts:
//   - valid sets verify true (single and aggregate, batchable and not);
//   - a wrong signature resolves false, a malformed one rejects with its BLST code, and neither affects
//     other concurrent calls (multithread.test.ts:89-106);
//   - more than 32 buffered batchable sets flush without waiting for the 100 ms timer;
//   - close() rejects buffered jobs with QUEUE_ERROR_QUEUE_ABORTED.
// Usage: BLSGPU_FAULT_INJECTION=1 node tests/node/verifier_gpu.js   (exit code 0 = pass; one line per check; without
// the variable the addon does not export debugInject and the fault-injection checks are skipped)
const assert = require("assert");
const fs = require("fs");
const path = require("path");

const ROOT = path.join(__dirname, "..", "..");
const {
  BlsGpuVerifier,
  BlsGpuSingleThreadVerifier,
  verifySignatureSet,
  fastAggregateVerify,
  ethFastAggregateVerify,
} = require(path.join(ROOT, "lodestar_amd", "node", "BlsGpuVerifier.cjs"));
const fx = JSON.parse(fs.readFileSync(path.join(ROOT, "tests", "golden", "verify_sets.json"), "utf8"));
const fav = JSON.parse(fs.readFileSync(path.join(ROOT, "tests", "golden", "fav_cases.json"), "utf8"));

// a PublicKey-like object (blst PublicKey.toBytes(PointFormat.uncompressed)), never registered
const pkObject = (bytes) => ({toBytes: () => bytes});

// metrics double: records every inc/observe/set by series name
function fakeMetrics() {
  const seen = {};
  const series = (name) => ({
    inc: (a, b) => (seen[name] = (seen[name] || 0) + (typeof a === "number" ? a : b === undefined ? 1 : b)),
    observe: (v) => (seen[name] = (seen[name] || 0) + 1),
    set: (v) => (seen[name] = v),
    addCollect: (fn) => fn(),
  });
  const names = ["jobsWorkerTime", "successJobsSignatureSetsCount", "errorJobsSignatureSetsCount", "jobWaitTime",
    "queueLength", "totalJobsGroupsStarted", "totalJobsStarted", "totalSigSetsStarted", "batchRetries",
    "batchSigsSuccess", "latencyToWorker", "latencyFromWorker", "mainThreadDurationInThreadPool", "timePerSigSet"];
  const blsThreadPool = {};
  for (const n of names) blsThreadPool[n] = series(n);
  return {seen, metrics: {blsThreadPool, bls: {aggregatedPubkeys: series("aggregatedPubkeys")}}};
}

const hex = (h) => Uint8Array.from(Buffer.from(h, "hex"));
const keys = fx.keys.map((k) => hex(k.pk));

function toSet(s, byIndex) {
  const msg = hex(s.msg);
  const sig = hex(s.sig);
  if (s.pks.length === 1 && !s.name.startsWith("aggregate")) {
    return {type: "single", pubkey: byIndex ? s.pks[0] : keys[s.pks[0]], signingRoot: msg, signature: sig};
  }
  return {type: "aggregate", pubkeys: s.pks.slice(), signingRoot: msg, signature: sig};
}

async function settle(p) {
  try {
    return {value: await p};
  } catch (e) {
    return {error: e};
  }
}

function expectOutcome(out, code, label, mainThread = false) {
  if (code === 1 || code === 0) {
    assert.ok(!out.error, `${label}: unexpected rejection ${out.error && out.error.message}`);
    assert.strictEqual(out.value, code === 1, `${label}: expected ${code === 1}`);
  } else {
    assert.ok(out.error, `${label}: expected rejection (code ${code}), got ${out.value}`);
    const want = {8: "BLST_INVALID_SIZE", 1: "BLST_BAD_ENCODING", 2: "BLST_POINT_NOT_ON_CURVE",
      3: "BLST_POINT_NOT_IN_GROUP", 9: "EMPTY_AGGREGATE_ARRAY",
      // an empty call: the pool ANDs no job results (index.ts:169-171), the main thread path throws in
      // verifySignatureSetsMaybeBatch (maybeBatch.ts:29-31)
      10: mainThread ? "Empty signature set" : "Empty results array"}[-code];
    assert.ok(out.error.message.includes(want), `${label}: message "${out.error.message}" lacks ${want}`);
  }
}

async function main() {
  const v = new BlsGpuVerifier({seed: 0x4c4f4445}, {});
  const table = Buffer.concat(keys.map((k) => Buffer.from(k)));
  v.uploadPubkeys(0, Uint8Array.from(table));

  // every golden case, each job as one concurrent verifySignatureSets call (table mode: indexed pubkeys)
  for (const c of fx.cases) {
    const outs = await Promise.all(
      c.jobs.map((j) => settle(v.verifySignatureSets(j.map((k) => toSet(fx.sets[k], true)), {batchable: c.batchable})))
    );
    outs.forEach((o, ji) => expectOutcome(o, c.expected[ji], `${c.name} job ${ji}`));
    console.log(`ok ${c.name} (${c.jobs.length} concurrent calls)`);
  }

  // bytes-mode pubkeys (what the pool sends its workers, index.ts:160): single sets only
  const singles = fx.cases.find((c) => c.name === "each_alone/batchable");
  const outs = await Promise.all(
    singles.jobs.map((j, ji) => {
      const s = fx.sets[j[0]];
      if (s.pks.length !== 1 || s.name.startsWith("aggregate")) return Promise.resolve(null);
      return settle(v.verifySignatureSets([toSet(s, false)], {batchable: true}));
    })
  );
  outs.forEach((o, ji) => o && expectOutcome(o, singles.expected[ji], `bytes-mode job ${ji}`));
  console.log("ok bytes-mode pubkeys");

  // > MAX_BUFFERED_SIGS batchable sets flush before the 100 ms timer
  const valid = fx.sets.slice(0, 8).map((s) => toSet(s, true));
  const t0 = Date.now();
  const many = [];
  for (let r = 0; r < 5; r++) for (const s of valid) many.push(v.verifySignatureSets([s], {batchable: true}));
  const res = await Promise.all(many);
  assert.ok(res.every((x) => x === true));
  console.log(`ok 40 buffered batchable calls in ${Date.now() - t0} ms, stats ${JSON.stringify(v.stats)}`);

  // verifyOnMainThread path (no buffering; BLSGPU_JOB_URGENT: the device's urgent lane, multithread/index.ts:138-151)
  const urgentBefore = v.stats.urgentCalls || 0;
  assert.strictEqual(await v.verifySignatureSets(valid.slice(0, 3), {verifyOnMainThread: true}), true);
  assert.strictEqual(await v.verifySignatureSets(valid.slice(3, 4), {verifyOnMainThread: true}), true);
  assert.strictEqual(v.stats.urgentCalls - urgentBefore, 2, "verifyOnMainThread calls ran on the urgent lane");
  // a batchable call is not urgent
  const urgentMid = v.stats.urgentCalls;
  assert.strictEqual(await v.verifySignatureSets(valid.slice(0, 1), {batchable: true}), true);
  assert.strictEqual(v.stats.urgentCalls, urgentMid);
  console.log("ok verifyOnMainThread (urgent lane)");

  // aggregate sets of plain PublicKey objects (no registration): bytes-aggregate mode on the GPU -- the gossip
  // attestation call (attestation.ts:131-138), every golden case
  for (const c of fx.cases) {
    const outs = await Promise.all(
      c.jobs.map((j) =>
        settle(
          v.verifySignatureSets(
            j.map((k) => {
              const s = fx.sets[k];
              return {type: "aggregate", pubkeys: s.pks.map((i) => pkObject(keys[i])), signingRoot: hex(s.msg),
                signature: hex(s.sig)};
            }),
            {batchable: c.batchable}
          )
        )
      )
    );
    outs.forEach((o, ji) => expectOutcome(o, c.expected[ji], `bytes-aggregate ${c.name} job ${ji}`));
  }
  console.log("ok aggregate sets of unregistered PublicKey objects (bytes-aggregate mode)");

  // empty calls: the pool path rejects "Empty results array" (index.ts:169-171), the main-thread path
  // "Empty signature set" (maybeBatch.ts:29-31)
  const e1 = await settle(v.verifySignatureSets([], {batchable: true}));
  assert.ok(e1.error && e1.error.message === "Empty results array", `empty pool call: ${e1.error}`);
  const e2 = await settle(v.verifySignatureSets([], {verifyOnMainThread: true}));
  assert.ok(e2.error && e2.error.message === "Empty signature set");
  console.log("ok empty calls");

  // 1,000-call gossip burst: one-pubkey aggregate sets of PublicKey objects, every 97th over a wrong root
  {
    const good = fx.sets.filter((s) => s.name.startsWith("single"));
    const calls = [];
    const want = [];
    for (let i = 0; i < 1000; i++) {
      const s = good[i % good.length];
      const bad = i % 97 === 5;
      const msg = hex(s.msg);
      if (bad) msg[0] ^= 1;
      calls.push(settle(v.verifySignatureSets(
        [{type: "aggregate", pubkeys: [pkObject(keys[s.pks[0]])], signingRoot: msg, signature: hex(s.sig)}],
        {batchable: true})));
      want.push(!bad);
    }
    const t0 = Date.now();
    const outs = await Promise.all(calls);
    outs.forEach((o, i) => {
      assert.ok(!o.error, `burst ${i}: ${o.error}`);
      assert.strictEqual(o.value, want[i], `burst ${i}`);
    });
    console.log(`ok 1000-call gossip burst in ${Date.now() - t0} ms (${want.filter((x) => !x).length} false)`);
  }

  // verifySignatureSet (signatureSets.ts:24-38) and the spec runner's fast_aggregate_verify entry points
  const agg = fx.sets.find((s) => s.name.startsWith("aggregate") && s.pks.length > 1);
  assert.strictEqual(await verifySignatureSet(v, {type: "aggregate", pubkeys: agg.pks.map((i) => keys[i]),
    signingRoot: hex(agg.msg), signature: hex(agg.sig)}), true);
  for (const c of fav.cases) {
    const pks = c.pubkeys.map(hex);
    assert.strictEqual(await fastAggregateVerify(v, pks, hex(c.message), hex(c.signature)), c.fast_aggregate_verify,
      `fast_aggregate_verify ${c.name}`);
    assert.strictEqual(await ethFastAggregateVerify(v, pks, hex(c.message), hex(c.signature)),
      c.eth_fast_aggregate_verify, `eth_fast_aggregate_verify ${c.name}`);
  }
  console.log(`ok verifySignatureSet + ${fav.cases.length} fast_aggregate_verify cases`);

  // a device failure rejects every job of the call with the device status, never `false` (index.ts:368-375), and
  // the verifier keeps serving: the next call verifies (fault injection: blsgpu_debug_inject)
  const {addon} = require(path.join(ROOT, "lodestar_amd", "node", "BlsGpuVerifier.cjs"));
  if (typeof addon.debugInject !== "function") {
    console.log("skip fault injection (run with BLSGPU_FAULT_INJECTION=1)");
  } else {
    addon.debugInject(2, 0, 1);
    const outs = await Promise.all([
      settle(v.verifySignatureSets(valid.slice(0, 3), {verifyOnMainThread: true})),
    ]);
    for (const o of outs)
      assert.ok(o.error && o.error.message.includes("BLSGPU_DEVICE_ERROR"), `device error: ${o.error || o.value}`);
    addon.debugInject(2, 0, 0);
    assert.strictEqual(await v.verifySignatureSets(valid.slice(0, 3), {verifyOnMainThread: true}), true);
    // production scalars (seed 0: a fresh OS key per call) and their fail-closed path
    const prod = new BlsGpuVerifier({}, {});
    prod.uploadPubkeys(0, Uint8Array.from(table));
    const c = fx.cases.find((x) => x.name === "multi_set_jobs/plain");
    const po = await Promise.all(c.jobs.map((j) => settle(prod.verifySignatureSets(j.map((k) => toSet(fx.sets[k], true)),
      {batchable: c.batchable}))));
    po.forEach((o, ji) => expectOutcome(o, c.expected[ji], `seed-0 ${c.name} job ${ji}`));
    addon.debugInject(1, 0, 1);
    const ent = await settle(prod.verifySignatureSets(valid.slice(0, 3), {verifyOnMainThread: true}));
    addon.debugInject(1, 0, 0);
    assert.ok(ent.error && ent.error.message.includes("BLSGPU_ERR_ENTROPY"), `entropy: ${ent.error || ent.value}`);
    assert.strictEqual(await prod.verifySignatureSets(valid.slice(0, 3), {verifyOnMainThread: true}), true);
    await prod.close();
    console.log("ok device error rejects (BLSGPU_DEVICE_ERROR), seed-0 scalars, entropy failure rejects");
  }

  // close() rejects what is still buffered, and later calls
  const pending = settle(v.verifySignatureSets([valid[0]], {batchable: true}));
  await v.close();
  const p = await pending;
  assert.ok(p.error && p.error.message === "QUEUE_ERROR_QUEUE_ABORTED", `close: ${p.error && p.error.message}`);
  const after = await settle(v.verifySignatureSets([valid[0]]));
  assert.ok(after.error && after.error.message === "QUEUE_ERROR_QUEUE_ABORTED");
  console.log("ok close");

  // BlsSingleThreadVerifier semantics + metrics of the pool series
  const {seen, metrics} = fakeMetrics();
  const st = new BlsGpuSingleThreadVerifier({seed: 7}, {metrics});
  st.uploadPubkeys(0, Uint8Array.from(table));
  const each = fx.cases.find((c) => c.name === "each_alone/plain");
  const so = await Promise.all(each.jobs.map((j) => settle(st.verifySignatureSets(j.map((k) => toSet(fx.sets[k], true))))));
  so.forEach((o, ji) => expectOutcome(o, each.expected[ji], `single-thread job ${ji}`, true));
  assert.ok(!st.stats.urgentCalls, "the single-thread verifier's calls share the pipeline, not the urgent lane");
  const se = await settle(st.verifySignatureSets([]));
  assert.ok(se.error && se.error.message === "Empty signature set");
  for (const n of ["totalJobsStarted", "totalSigSetsStarted", "jobsWorkerTime", "timePerSigSet", "jobWaitTime",
    "successJobsSignatureSetsCount", "errorJobsSignatureSetsCount", "latencyToWorker"])
    assert.ok(seen[n] > 0, `metric ${n} not fed`);
  await st.close();
  console.log(`ok single-thread verifier, metrics ${JSON.stringify(seen)}`);
  console.log("ALL OK");
}

main().catch((e) => {
  console.error(e);
  process.exit(1);
});

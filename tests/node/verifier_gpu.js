"use strict";
// GPU parity of the JS drop-in (lodestar_amd/node/BlsGpuVerifier.js) against tests/golden/verify_sets.json,
// mirroring the reference's packages/beacon-node/test/e2e/chain/bls/multithread.test.ts:
//   - valid sets verify true (single and aggregate, batchable and not);
//   - a wrong signature resolves false, a malformed one rejects with its BLST code, and neither affects
//     other concurrent calls (multithread.test.ts:89-106);
//   - more than 32 buffered batchable sets flush without waiting for the 100 ms timer;
//   - close() rejects buffered jobs with QUEUE_ERROR_QUEUE_ABORTED.
// Usage: node tests/node/verifier_gpu.js   (exit code 0 = pass; prints one line per check)
const assert = require("assert");
const fs = require("fs");
const path = require("path");

const ROOT = path.join(__dirname, "..", "..");
const {BlsGpuVerifier} = require(path.join(ROOT, "lodestar_amd", "node", "BlsGpuVerifier.js"));
const fx = JSON.parse(fs.readFileSync(path.join(ROOT, "tests", "golden", "verify_sets.json"), "utf8"));

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

function expectOutcome(out, code, label) {
  if (code === 1 || code === 0) {
    assert.ok(!out.error, `${label}: unexpected rejection ${out.error && out.error.message}`);
    assert.strictEqual(out.value, code === 1, `${label}: expected ${code === 1}`);
  } else {
    assert.ok(out.error, `${label}: expected rejection (code ${code}), got ${out.value}`);
    const want = {8: "BLST_INVALID_SIZE", 1: "BLST_BAD_ENCODING", 2: "BLST_POINT_NOT_ON_CURVE",
      3: "BLST_POINT_NOT_IN_GROUP", 9: "EMPTY_AGGREGATE_ARRAY", 10: "Empty signature set"}[-code];
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

  // verifyOnMainThread path (no buffering)
  assert.strictEqual(await v.verifySignatureSets(valid.slice(0, 3), {verifyOnMainThread: true}), true);
  console.log("ok verifyOnMainThread");

  // close() rejects what is still buffered, and later calls
  const pending = settle(v.verifySignatureSets([valid[0]], {batchable: true}));
  await v.close();
  const p = await pending;
  assert.ok(p.error && p.error.message === "QUEUE_ERROR_QUEUE_ABORTED", `close: ${p.error && p.error.message}`);
  const after = await settle(v.verifySignatureSets([valid[0]]));
  assert.ok(after.error && after.error.message === "QUEUE_ERROR_QUEUE_ABORTED");
  console.log("ok close");
  console.log("ALL OK");
}

main().catch((e) => {
  console.error(e);
  process.exit(1);
});

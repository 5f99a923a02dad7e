// The drop-in as the ES-module beacon-node package loads it (reference packages/beacon-node/package.json:15
// "type": "module"): import the ESM entry, check the IBlsVerifier surface (interface.ts:20-46), then construct a
// verifier.  On a GPU box it verifies one reference-shaped set (multithread.test.ts:28-41 style keys are in the
// golden fixture) and closes; without a GPU the constructor must fail loudly (no CPU fallback).
// Usage: node tests/node/esm_entry.mjs   -> prints one JSON line
import fs from "fs";
import path from "path";
import {fileURLToPath} from "url";

import def, {BlsGpuVerifier, BlsGpuSingleThreadVerifier, verifySignatureSet, fastAggregateVerify, QueueError}
  from "../../lodestar_amd/node/index.js";

const here = path.dirname(fileURLToPath(import.meta.url));
const out = {esm: true, exports: []};
for (const [k, v] of Object.entries({BlsGpuVerifier, BlsGpuSingleThreadVerifier, verifySignatureSet, fastAggregateVerify, QueueError}))
  if (typeof v === "function") out.exports.push(k);
if (def.BlsGpuVerifier !== BlsGpuVerifier) throw new Error("default export mismatch");
for (const m of ["verifySignatureSets", "close"])
  if (typeof BlsGpuVerifier.prototype[m] !== "function") throw new Error("IBlsVerifier method missing: " + m);

let v = null;
try {
  v = new BlsGpuVerifier({seed: 7}, {});
} catch (e) {
  out.threw = e.message;
}
async function main() {
  if (!v) return;
  const fx = JSON.parse(fs.readFileSync(path.join(here, "..", "golden", "verify_sets.json"), "utf8"));
  const hex = (h) => Uint8Array.from(Buffer.from(h, "hex"));
  const keys = fx.keys.map((k) => hex(k.pk));
  out.hwQueues = v.getOption("hw_queues");
  out.slots = v.getOption("slots");
  const s = fx.sets.find((x) => x.pks.length === 1 && x.sig.length === 192);
  const set = {type: "single", pubkey: keys[s.pks[0]], signingRoot: hex(s.msg), signature: hex(s.sig)};
  out.verified = await v.verifySignatureSets([set], {batchable: true});
  await v.close();
  try {
    await v.verifySignatureSets([set]);
  } catch (e) {
    out.afterClose = e.message;
  }
}
main().then(
  () => console.log(JSON.stringify(out)),
  (e) => {
    console.error(e);
    process.exit(1);
  }
);

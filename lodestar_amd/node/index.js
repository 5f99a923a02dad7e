// ESM entry of the IBlsVerifier drop-in.  packages/beacon-node is an ES module package (reference
// packages/beacon-node/package.json:15 "type": "module"), so chain.ts imports this file:
//   import {BlsGpuVerifier} from "./bls/gpu/index.js";
// The implementation is CommonJS (BlsGpuVerifier.cjs: it loads the N-API addon with require); createRequire bridges
// the two module systems without a build step (Node >= 12.2).
import {createRequire} from "module";

const require = createRequire(import.meta.url);
const impl = require("./BlsGpuVerifier.cjs");

export const {
  BlsGpuVerifier,
  BlsGpuSingleThreadVerifier,
  verifySignatureSet,
  fastAggregateVerify,
  ethFastAggregateVerify,
  QueueError,
  SignatureSetType,
  MAX_BUFFERED_SIGS,
  MAX_BUFFER_WAIT_MS,
  addon,
} = impl;
export default impl;

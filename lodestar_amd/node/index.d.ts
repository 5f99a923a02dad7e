// Types of the IBlsVerifier drop-in, for packages/beacon-node/src/chain/bls/gpu/ (next to interface.ts, reference
// packages/beacon-node/src/chain/bls/interface.ts:20-46, and the ISignatureSet union of
// state-transition/src/util/signatureSets.ts:10-22).
import type {ISignatureSet} from "@lodestar/state-transition";
import type {IBlsVerifier, VerifySignatureOpts} from "../interface.js";

/** A set's pubkey as the drop-in takes it: a validator index into the device table (uploadPubkeys), a PublicKey
 * registered with registerPubkey, any object serializing to 96 uncompressed bytes (blst PublicKey.toBytes()), or
 * those bytes. */
export type GpuPubkey = number | Uint8Array | {toBytes(format?: unknown): Uint8Array};

export type BlsGpuVerifierOpts = {
  /** HIP devices to shard calls over (default: every visible device) */
  devices?: number[];
  /** sets per batch group (default 1024) */
  groupSets?: number;
  /** 0 = batch groups of >= groupSets sets (default); 1 = the pool's jobs / requests / >= 16-job chunks, so the
   * batchRetries / batchSigsSuccess metrics count the reference's units */
  groupPolicy?: 0 | 1;
  /** batch-scalar seed for comparison runs; 0 / undefined = OS CSPRNG */
  seed?: number;
};

export type BlsGpuVerifierModules = {
  metrics?: unknown | null;
  logger?: unknown;
};

export declare class QueueError extends Error {
  type: {code: string};
}

export declare class BlsGpuVerifier implements IBlsVerifier {
  constructor(opts?: BlsGpuVerifierOpts, modules?: BlsGpuVerifierModules);
  /** IBlsVerifier.verifySignatureSets: true iff every set verifies; rejects with "BLST_ERROR: <CODE>" where the
   * reference's Signature.fromBytes throws, "QUEUE_ERROR_QUEUE_ABORTED" once closed. */
  verifySignatureSets(sets: ISignatureSet[], opts?: VerifySignatureOpts): Promise<boolean>;
  /** IBlsVerifier.close: rejects buffered jobs with QUEUE_ERROR_QUEUE_ABORTED, then frees the devices. */
  close(): Promise<void>;
  /** index2pubkey sync: entries [firstIndex, firstIndex + n) as 96-byte uncompressed encodings. */
  uploadPubkeys(firstIndex: number, pk96: Uint8Array): void;
  /** maps a PublicKey object (by identity) to its validator index in the device table */
  registerPubkey(pk: object, index: number): void;
  readonly deviceCount: number;
  /** a runtime tunable or property: "slots", "hw_queues", "group_sets", "group_policy", "merge_sets", ... */
  getOption(key: string): number;
}

export declare class BlsGpuSingleThreadVerifier extends BlsGpuVerifier {}

export declare function verifySignatureSet(verifier: BlsGpuVerifier, set: ISignatureSet): Promise<boolean>;
export declare function fastAggregateVerify(
  verifier: BlsGpuVerifier,
  pubkeys48: Uint8Array[],
  message: Uint8Array,
  signature: Uint8Array
): Promise<boolean>;
export declare function ethFastAggregateVerify(
  verifier: BlsGpuVerifier,
  pubkeys48: Uint8Array[],
  message: Uint8Array,
  signature: Uint8Array
): Promise<boolean>;

export declare const SignatureSetType: {single: "single"; aggregate: "aggregate"};
export declare const MAX_BUFFERED_SIGS: number;
export declare const MAX_BUFFER_WAIT_MS: number;
export declare const addon: Record<string, (...args: unknown[]) => unknown>;

// (f4) Signing-root production: SSZ hash_tree_root of SigningData{object_root, domain} and of AttestationData,
// the step before the verifier on block import and gossip (reference state-transition/src/util/
// signingRoot.ts:7-13 computeSigningRoot; consensus-specs phase0 AttestationData / Checkpoint / SigningData).
// One lane per object; SHA-256 compressions from hash_to_curve.hpp.
#include "k_common.hpp"

// SHA-256 of a 64-byte message given as 16 big-endian words -> 8 state words
__device__ void sha256_64(const uint32_t in[16], uint32_t out[8]) {
  sha_st st;
#pragma unroll
  for (int i = 0; i < 8; i++) st.h[i] = SHA256_IV[i];
  st = sha256_block(st, sha_blk_of(in));
  sha_blk pad;
#pragma unroll
  for (int i = 0; i < 16; i++) pad.w[i] = 0;
  pad.w[0] = 0x80000000u;
  pad.w[15] = 512u;
  st = sha256_block(st, pad);
#pragma unroll
  for (int i = 0; i < 8; i++) out[i] = st.h[i];
}

__device__ __forceinline__ uint32_t be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
// a 32-byte chunk holding a little-endian uint64 (SSZ basic type), as big-endian words
__device__ __forceinline__ void u64_chunk(const uint8_t* le8, uint32_t* w) {
  w[0] = be32(le8);
  w[1] = be32(le8 + 4);
#pragma unroll
  for (int i = 2; i < 8; i++) w[i] = 0;
}
__device__ __forceinline__ void bytes_chunk(const uint8_t* b32, uint32_t* w) {
#pragma unroll
  for (int i = 0; i < 8; i++) w[i] = be32(b32 + 4 * i);
}
__device__ __forceinline__ void hash_pair(const uint32_t* a, const uint32_t* b, uint32_t* out) {
  uint32_t blk[16];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    blk[i] = a[i];
    blk[8 + i] = b[i];
  }
  sha256_64(blk, out);
}
// Checkpoint{epoch, root} (serialized: epoch LE 8 B, root 32 B)
__device__ void checkpoint_root(const uint8_t* cp, uint32_t* out) {
  uint32_t e[8], r[8];
  u64_chunk(cp, e);
  bytes_chunk(cp + 8, r);
  hash_pair(e, r, out);
}

// kind 0: in = object_root (32 B);  kind 1: in = serialized AttestationData (128 B):
//   slot u64 | index u64 | beacon_block_root 32 | source {epoch u64, root 32} | target {epoch u64, root 32}
// out = hash_tree_root(SigningData{hash_tree_root(object), domain})
__global__ __launch_bounds__(WAVE) void k_signing_roots(int kind, const uint8_t* in, uint32_t n, uint32_t in_stride,
                                                        const uint8_t* domain, uint32_t domain_stride, uint8_t* out) {
  const uint32_t i = blockIdx.x * WAVE + threadIdx.x;
  if (i >= n) return;
  const uint8_t* o = in + (size_t)i * in_stride;
  uint32_t root[8];
  if (kind == 0) {
    bytes_chunk(o, root);
  } else {
    uint32_t leaf[5][8], zero[8], l1[4][8], l2[2][8];
    u64_chunk(o, leaf[0]);
    u64_chunk(o + 8, leaf[1]);
    bytes_chunk(o + 16, leaf[2]);
    checkpoint_root(o + 48, leaf[3]);
    checkpoint_root(o + 88, leaf[4]);
#pragma unroll
    for (int k = 0; k < 8; k++) zero[k] = 0;
    hash_pair(leaf[0], leaf[1], l1[0]);
    hash_pair(leaf[2], leaf[3], l1[1]);
    hash_pair(leaf[4], zero, l1[2]);
    uint32_t zz[8];
    hash_pair(zero, zero, zz);
    hash_pair(l1[0], l1[1], l2[0]);
    hash_pair(l1[2], zz, l2[1]);
    hash_pair(l2[0], l2[1], root);
  }
  uint32_t d[8], sr[8];
  bytes_chunk(domain + (size_t)i * domain_stride, d);
  hash_pair(root, d, sr);
  uint8_t* dst = out + (size_t)i * 32;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    dst[4 * k] = (uint8_t)(sr[k] >> 24);
    dst[4 * k + 1] = (uint8_t)(sr[k] >> 16);
    dst[4 * k + 2] = (uint8_t)(sr[k] >> 8);
    dst[4 * k + 3] = (uint8_t)sr[k];
  }
}

void launch_signing_roots(int kind, const uint8_t* in, uint32_t n, uint32_t in_stride, const uint8_t* domain,
                          uint32_t domain_stride, uint8_t* out, hipStream_t s) {
  if (n)
    hipLaunchKernelGGL(k_signing_roots, dim3((n + WAVE - 1) / WAVE), dim3(WAVE), 0, s, kind, in, n, in_stride,
                       domain, domain_stride, out);
}

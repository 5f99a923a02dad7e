// Batch scalars of the random linear combination (host side, runtime.cpp).
//
// The reference draws blst's 64-bit scalars from fresh randomness in every verifyMultipleAggregateSignatures call
// (chain/bls/maybeBatch.ts:17-26 -> blst; SURVEY.md §7 hard part 5): an attacker who could predict them could build
// invalid sets whose defects cancel in the combination.  Here each call gets a 256-bit ChaCha20 key and scalar word i
// of the call is 64 bits of the ChaCha20 keystream (RFC 8439 block function, block i / 8, words 2 (i % 8) and
// 2 (i % 8) + 1):
//   * seed == 0 (production): the key is 32 bytes of getrandom(2) (retried on EINTR and short reads).  If the OS
//     cannot provide them the call FAILS (BLSGPU_ERR_ENTROPY): there is no constant or time-based fallback.
//   * seed != 0 (comparison runs only): the key is the seed under a fixed domain constant -- deterministic, so GPU
//     and oracle runs can be repeated; never the production path.
// Word 0 encodes r = 1 (CoreVerify of a lone non-batchable set), so a keystream word of 0 becomes 1.
#pragma once
#include <errno.h>
#include <stdint.h>
#include <string.h>
#include <sys/random.h>

#include <atomic>

namespace batch_rand {

struct Key {
  uint32_t k[8];
};

inline uint32_t rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

#define BR_QR(a, b, c, d)   \
  a += b, d ^= a, d = rotl(d, 16); \
  c += d, b ^= c, b = rotl(b, 12); \
  a += b, d ^= a, d = rotl(d, 8);  \
  c += d, b ^= c, b = rotl(b, 7)

// One ChaCha20 block (RFC 8439 §2.3): key, 32-bit block counter, 96-bit nonce.  Every key serves one call; the nonce
// separates the keystreams a call draws: nonce 0 = the batch scalar words, kNonceHashKey = the message index's hash key.
constexpr uint32_t kNonceHashKey = 0x68736b31u;  // "1ksh"
inline void chacha20_block(const Key& key, uint32_t counter, uint32_t out[16], uint32_t nonce0 = 0) {
  uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, key.k[0], key.k[1], key.k[2], key.k[3],
                    key.k[4],    key.k[5],    key.k[6],    key.k[7],    counter,  nonce0,   0u,       0u};
  uint32_t x[16];
  memcpy(x, s, sizeof x);
  for (int r = 0; r < 10; r++) {
    BR_QR(x[0], x[4], x[8], x[12]);
    BR_QR(x[1], x[5], x[9], x[13]);
    BR_QR(x[2], x[6], x[10], x[14]);
    BR_QR(x[3], x[7], x[11], x[15]);
    BR_QR(x[0], x[5], x[10], x[15]);
    BR_QR(x[1], x[6], x[11], x[12]);
    BR_QR(x[2], x[7], x[8], x[13]);
    BR_QR(x[3], x[4], x[9], x[14]);
  }
  for (int i = 0; i < 16; i++) out[i] = x[i] + s[i];
}
#undef BR_QR

// Test hook (blsgpu_debug_inject): the next `count` entropy draws after `skip` more fail as if getrandom did.
inline std::atomic<int64_t>& inject_skip() {
  static std::atomic<int64_t> v{0};
  return v;
}
inline std::atomic<int64_t>& inject_count() {
  static std::atomic<int64_t> v{0};
  return v;
}
// Consumes one event of an armed (skip, count) injection: true = this event fails.
inline bool take_injection(std::atomic<int64_t>& skip, std::atomic<int64_t>& count) {
  for (;;) {
    int64_t c = count.load();
    if (c <= 0) return false;
    int64_t s = skip.load();
    if (s > 0) {
      if (skip.compare_exchange_weak(s, s - 1)) return false;
      continue;
    }
    if (count.compare_exchange_weak(c, c - 1)) return true;
  }
}

// 32 bytes of OS entropy into key; false when the OS cannot provide them (the call must then fail).
inline bool os_key(Key& key) {
  if (take_injection(inject_skip(), inject_count())) return false;
  uint8_t* p = reinterpret_cast<uint8_t*>(key.k);
  size_t got = 0;
  while (got < sizeof key.k) {
    const ssize_t r = getrandom(p + got, sizeof key.k - got, 0);
    if (r > 0) {
      got += (size_t)r;
    } else if (r < 0 && errno == EINTR) {
      continue;
    } else {
      memset(key.k, 0, sizeof key.k);
      return false;
    }
  }
  return true;
}

// Comparison-run key: the seed under a domain constant ("lodestar-amd batch scalar keys").
inline Key seed_key(uint64_t seed) {
  return Key{{(uint32_t)seed, (uint32_t)(seed >> 32), 0x65646f6cu, 0x72617473u, 0x646d612du, 0x61637320u,
              0x2072616cu, 0x7379656bu}};
}

// The message index's hash key (runtime.cpp MsgIndex): 64 bits of the call key's own keystream under a separate nonce,
// so no key word of the scalars' keystream ever drives the host hash table (a timing leak of the table would reveal
// nothing about the scalars).
inline uint64_t hash_key(const Key& key) {
  uint32_t blk[16];
  chacha20_block(key, 0, blk, kNonceHashKey);
  return (uint64_t)blk[0] | ((uint64_t)blk[1] << 32);
}

// Scalar words [first, first + n) of the call keyed by `key` -> out[0 .. n)
inline void words(const Key& key, uint64_t first, uint64_t n, uint64_t* out) {
  uint32_t blk[16];
  uint64_t cur = UINT64_MAX;
  for (uint64_t t = 0; t < n; t++) {
    const uint64_t i = first + t;
    if (i / 8 != cur) {
      cur = i / 8;
      chacha20_block(key, (uint32_t)cur, blk);
    }
    const int j = (int)(i % 8);
    const uint64_t w = (uint64_t)blk[2 * j] | ((uint64_t)blk[2 * j + 1] << 32);
    out[t] = w ? w : 1;
  }
}

}  // namespace batch_rand

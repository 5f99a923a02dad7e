/* TEST INFRASTRUCTURE ONLY: self-test of the C restatement, built with ASan + UBSan by `make -C oracle
 * sanitize` (tests/test_cpu_oracle.py).  Exercises every entry point on the reference's deposit KAT
 * (beacon-node/test/e2e/interop/genesisState.test.ts:51-55) and a small pool run with an invalid set. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "blscpu.h"

static void unhex(const char* h, uint8_t* out) {
  for (size_t i = 0; h[2 * i]; i++) {
    unsigned v;
    sscanf(h + 2 * i, "%2x", &v);
    out[i] = (uint8_t)v;
  }
}
#define CHECK(c)                                         \
  do {                                                   \
    if (!(c)) {                                          \
      fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c); \
      return 1;                                          \
    }                                                    \
  } while (0)

int main(void) {
  uint8_t sk[32], root[32], pk48[48], sig[96], pk96[96], s2[96];
  unhex("25295f0d1d592a90b333e26e85149708208e9f8e8bc18f6c77bd62f8ad7a6866", sk);
  unhex("f9e9adcff9c1517685beae7922ba8d8743626199d2bd7b397f3bd97ac140b542", root);
  unhex("a99a76ed7796f7be22d5b7e85deeb7c5677e88e511e0b337618f8c4eb61349b4bf2d153f649f7b53359fe8b94a38e44c", pk48);
  unhex("a95af8ff0f8c06af4d29aef05ce865f85f82df42b606008ec5b1bcb42b17ae47f4b78cdce1db31ce32d18f42a6b296b4"
        "014a2164981780e56b5a40d7723c27b8423173e58fa36f075078b177634f66351412b867c103f532aedd50bcd9b98446",
        sig);
  CHECK(blscpu_sk_to_pk(1, sk, pk96, 1) == 0);
  uint8_t dec[96];
  CHECK(blscpu_pk_decode(pk48, 48, dec) == 0 && memcmp(dec, pk96, 96) == 0);
  CHECK(blscpu_key_validate(pk48, 48) == 0);
  CHECK(blscpu_sign(1, sk, root, s2, 1) == 0 && memcmp(s2, sig, 96) == 0);
  CHECK(blscpu_sig_status(sig, 96) == 0);

  /* 20 sets: the deposit set repeated, set 7 over a wrong root; jobs of 1 set, batchable */
  enum { N = 20 };
  uint8_t msgs[32 * N], sigs[96 * N], pks[96 * N];
  uint32_t jfs[N + 1], sl[N];
  uint8_t flags[N];
  for (int i = 0; i < N; i++) {
    memcpy(msgs + 32 * i, root, 32);
    memcpy(sigs + 96 * i, sig, 96);
    memcpy(pks + 96 * i, pk96, 96);
    jfs[i] = (uint32_t)i;
    sl[i] = 96;
    flags[i] = 1;
  }
  jfs[N] = N;
  msgs[32 * 7] ^= 1;
  blsgpu_batch b;
  memset(&b, 0, sizeof b);
  b.n_sets = N;
  b.n_jobs = N;
  b.job_first_set = jfs;
  b.job_flags = flags;
  b.pk_bytes = pks;
  b.msgs = msgs;
  b.sigs = sigs;
  b.sig_len = sl;
  b.sig_stride = 96;
  b.seed = 42;
  int8_t res[N];
  blscpu_stats st;
  CHECK(blscpu_verify_jobs(&b, NULL, res, 4, &st) == 0);
  for (int i = 0; i < N; i++) CHECK(res[i] == (i == 7 ? 0 : 1));
  CHECK(st.batch_retries == 1);

  /* table mode aggregate of 3 copies */
  blscpu_table* t = blscpu_table_create(pk96, 1, NULL);
  CHECK(t != NULL);
  uint32_t spf[2] = {0, 3}, idx[3] = {0, 0, 0}, jf1[2] = {0, 1};
  blsgpu_batch a;
  memset(&a, 0, sizeof a);
  a.n_sets = 1;
  a.n_jobs = 1;
  a.job_first_set = jf1;
  a.set_pk_first = spf;
  a.pk_index = idx;
  a.msgs = msgs;
  a.sigs = sigs;
  a.sig_len = sl;
  a.sig_stride = 96;
  uint8_t agg[96];
  int8_t ast;
  CHECK(blscpu_aggregate_pubkeys(&a, t, agg, 96, &ast, 1) == 0 && ast == 0);
  blscpu_table_free(t);
  printf("selftest ok\n");
  return 0;
}

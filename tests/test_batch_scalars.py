"""CPU tests of the batch scalars (random linear combination) through the C-ABI's pure host entry
blsgpu_batch_scalars: ChaCha20 keystream words (lodestar_amd/csrc/batch_rand.hpp), pinned here by an independent
Python ChaCha20 checked against the RFC 8439 §2.3.2 block vector; seed 0 draws fresh OS entropy per call and fails
closed (BLSGPU_ERR_ENTROPY) when the entropy source fails (fault-injection hook).  The reference draws blst's scalars
from fresh randomness per verifyMultipleAggregateSignatures call (chain/bls/maybeBatch.ts:17-26)."""
import os
import struct

import numpy as np
import pytest

from lodestar_amd import native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rotl(x, r):
    return ((x << r) | (x >> (32 - r))) & 0xFFFFFFFF


def chacha20_block(key_words, counter, nonce_words=(0, 0, 0)):
    s = [0x61707865, 0x3320646E, 0x79622D32, 0x6B206574, *key_words, counter, *nonce_words]
    x = list(s)

    def qr(a, b, c, d):
        x[a] = (x[a] + x[b]) & 0xFFFFFFFF; x[d] = _rotl(x[d] ^ x[a], 16)
        x[c] = (x[c] + x[d]) & 0xFFFFFFFF; x[b] = _rotl(x[b] ^ x[c], 12)
        x[a] = (x[a] + x[b]) & 0xFFFFFFFF; x[d] = _rotl(x[d] ^ x[a], 8)
        x[c] = (x[c] + x[d]) & 0xFFFFFFFF; x[b] = _rotl(x[b] ^ x[c], 7)

    for _ in range(10):
        qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15)
        qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14)
    return [(x[i] + s[i]) & 0xFFFFFFFF for i in range(16)]


def test_python_chacha20_matches_rfc8439_block_vector():
    key = struct.unpack("<8I", bytes(range(32)))
    nonce = struct.unpack("<3I", bytes.fromhex("000000090000004a00000000"))
    out = chacha20_block(key, 1, nonce)
    want = bytes.fromhex(
        "10f1e7e4d13b5915500fdd1fa32071c4c7d1f4c733c068030422aa9ac3d46c4e"
        "d2826446079faa0914c2d705d98b02a2b5129cd1de164eb9cbd083e8a2503c4e")
    assert struct.pack("<16I", *out) == want


def seed_key(seed):
    # batch_rand.hpp seed_key: the seed under the domain constant "lodestar-amd batch scalar keys"
    return [seed & 0xFFFFFFFF, seed >> 32, 0x65646F6C, 0x72617473, 0x646D612D, 0x61637320, 0x2072616C, 0x7379656B]


def expected_words(jfs, flags, seed):
    n = jfs[-1]
    key = seed_key(seed)
    out = []
    for i in range(n):
        blk = chacha20_block(key, i // 8)
        w = blk[2 * (i % 8)] | (blk[2 * (i % 8) + 1] << 32)
        out.append(w or 1)
    for j in range(len(jfs) - 1):
        if not (flags[j] & 1) and jfs[j + 1] - jfs[j] == 1:
            out[jfs[j]] = 0  # r = 1: CoreVerify of a lone non-batchable set
    return out


def test_fixed_seed_words_are_the_chacha20_keystream():
    jfs = [0, 1, 4, 5, 5, 37, 38]
    flags = [0, 1, 1, 0, 1, 0]
    for seed in (1, 0x4C4F444553544152, 2**64 - 1):
        got = native.batch_scalars(jfs, flags, seed)
        assert [int(x) for x in got] == expected_words(jfs, flags, seed)
    a = native.batch_scalars(jfs, flags, 7)
    b = native.batch_scalars(jfs, flags, 8)
    assert (a[1:4] != b[1:4]).all()


def test_seed_zero_draws_fresh_keys():
    jfs = np.arange(0, 4097, dtype=np.uint32)  # 4096 single-set batchable jobs
    flags = np.ones(4096, np.uint8)
    a = native.batch_scalars(jfs, flags, 0)
    b = native.batch_scalars(jfs, flags, 0)
    assert (a != 0).all() and (b != 0).all()
    assert len(set(a.tolist())) == 4096
    assert (a != b).sum() == 4096  # a new 256-bit key per call
    # roughly uniform 64-bit words: each bit set about half the time
    bits = np.unpackbits(a.view(np.uint8)).mean()
    assert 0.48 < bits < 0.52


def test_entropy_failure_fails_closed():
    jfs, flags = [0, 2, 3], [1, 0]
    native.debug_inject(native.INJECT_ENTROPY, 0, 1)
    try:
        with pytest.raises(RuntimeError, match="ERR_ENTROPY"):
            native.batch_scalars(jfs, flags, 0)
    finally:
        native.debug_inject(native.INJECT_ENTROPY, 0, 0)
    # fixed seeds never touch the entropy source; the next seed-0 call draws again
    native.debug_inject(native.INJECT_ENTROPY, 0, 1)
    try:
        assert len(native.batch_scalars(jfs, flags, 5)) == 3
        with pytest.raises(RuntimeError, match="ERR_ENTROPY"):
            native.batch_scalars(jfs, flags, 0)
        assert (native.batch_scalars(jfs, flags, 0)[:2] != 0).all()
    finally:
        native.debug_inject(native.INJECT_ENTROPY, 0, 0)
    assert native.code_name(native.ERR_ENTROPY) == "BLSGPU_ERR_ENTROPY"


def test_no_constant_scalar_fallback_in_runtime():
    """The runtime has no public-constant or counter fallback for production scalars (the round-3 SEED fallback)."""
    src = open(os.path.join(ROOT, "lodestar_amd", "csrc", "runtime.cpp")).read()
    src += open(os.path.join(ROOT, "lodestar_amd", "csrc", "batch_rand.hpp")).read()
    assert "4c4f444553544152" not in src.lower()
    assert "splitmix" not in src.lower()


def _raw_batch_scalars(jfs, n_sets, n_jobs=None):
    """blsgpu_batch_scalars on a raw job list (no Python-side checks): (rc, words)."""
    import ctypes

    jfs = np.ascontiguousarray(jfs, dtype=np.uint32)
    b = native.Batch()
    b.n_sets = n_sets
    b.n_jobs = len(jfs) - 1 if n_jobs is None else n_jobs
    b.job_first_set = jfs.ctypes.data
    b.seed = 3
    guard = np.full(max(n_sets, 1) + 16, 0xABABABABABABABAB, np.uint64)  # canaries past n_sets
    rc = native.load().blsgpu_batch_scalars(ctypes.byref(b), guard.ctypes.data)
    return rc, guard


@pytest.mark.parametrize("jfs,n_sets", [
    ([0, 5, 6, 3], 3),      # non-monotone: a single-set job would write words[5]
    ([1, 2, 3], 3),         # does not start at 0
    ([0, 2, 4], 3),         # does not end at n_sets
    ([0], 2),               # no jobs but sets
])
def test_batch_scalars_rejects_malformed_jobs(jfs, n_sets):
    """blsgpu_batch_scalars applies validate_batch's job_first_set rules before writing any word."""
    rc, guard = _raw_batch_scalars(jfs, n_sets)
    assert rc == native.ERR_ARGS
    assert (guard == 0xABABABABABABABAB).all()  # nothing written


def test_batch_scalars_python_rejects_empty_job_list():
    with pytest.raises(ValueError):
        native.batch_scalars(np.zeros(0, np.uint32))


def test_batch_scalars_accepts_empty_jobs():
    rc, guard = _raw_batch_scalars([0, 0, 2, 2, 3], 3)
    assert rc == native.OK
    assert (guard[3:] == 0xABABABABABABABAB).all()


def test_hash_key_is_not_scalar_key_material():
    """the message index's hash key is its own ChaCha20 block (nonce "1ksh"), not key words of the scalar
    keystream's key (batch_rand.hpp hash_key, runtime.cpp resolve_key)."""
    src = open(os.path.join(ROOT, "lodestar_amd", "csrc", "runtime.cpp")).read()
    assert "key.k[6]" not in src and "key.k[7]" not in src
    assert "batch_rand::hash_key(key)" in src


def test_fault_injection_needs_the_environment_switch():
    """blsgpu_debug_inject is armed only in a process started with BLSGPU_FAULT_INJECTION=1."""
    import subprocess
    import sys

    code = ("from lodestar_amd import native\n"
            "import sys\n"
            "try:\n"
            "    native.debug_inject(native.INJECT_ENTROPY, 0, 1)\n"
            "except ValueError:\n"
            "    sys.exit(7)\n"
            "sys.exit(0)\n")
    env = {k: v for k, v in os.environ.items() if k != "BLSGPU_FAULT_INJECTION"}
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env)
    assert r.returncode == 7
    env["BLSGPU_FAULT_INJECTION"] = "1"
    r = subprocess.run([sys.executable, "-c", code + ""], cwd=ROOT, env=env)
    assert r.returncode == 0

"""GPU parity at BASELINE.json's configs C3, C4 (one rank's shard and the whole 32,768-set step) and C5, job for job
against the C restatement of the reference pool (oracle/blscpu.c verify_jobs, pinned by tests/test_cpu_oracle.py)
on ORACLE-signed inputs: the workloads come from bench.py's generators with every signature made by
the oracle, and ~1% of the sets are corrupted in every way the reference distinguishes (oracle/corrupt.py).  Both
grouping policies run: the default >= 1,024-set groups and the reference pool's jobs / requests / chunks
(group_policy 1), whose batchRetries / batchSigsSuccess metrics must equal the oracle's."""
import os

import numpy as np
import pytest

import bench
from oracle import corrupt, cpu

pytestmark = pytest.mark.gpu

THREADS = bench.host_cpus()["threads"]


def oracle_sign(sks, msgs):
    return cpu.sign(sks, msgs, threads=THREADS)


@pytest.fixture(scope="module")
def ctx():
    from lodestar_amd.native import Context

    c = Context([0])
    yield c
    c.close()


def call_of(w, **over):
    call = {k: v for k, v in w.items() if k != "expected" and not k.startswith("_")}
    call.update(over)
    return call


def corrupted(w, seed):
    """The workload's sets re-signed by the oracle over fresh roots, ~1% corrupted (every class)."""
    n = len(w["_mkey"])
    msgs = [bench.msg_j(k, seed) for k in w["_mkey"]]
    sigs = cpu.sign(b"".join(w["_sk"]), b"".join(msgs), threads=THREADS)
    msgs, buf, sl, applied = corrupt.corrupt_sets([sigs[96 * i: 96 * i + 96] for i in range(n)], msgs,
                                                  np.random.default_rng(seed & 0xFFFF))
    return call_of(w, sigs=np.frombuffer(buf, np.uint8), sig_len=np.asarray(sl, np.uint32),
                   msgs=np.frombuffer(b"".join(msgs), np.uint8), sig_stride=192), applied


def compare(ctx, call, table, seed=bench.SEED, policy=0):
    ctx.set_option("group_policy", policy)
    try:
        got, st = ctx.verify_raw(**call, seed=seed)
    finally:
        ctx.set_option("group_policy", 0)
    want, ost = cpu.verify_jobs(table=table, threads=THREADS, **call, seed=seed)
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, f"{len(bad)} mismatches, first {bad[:8]}: got {got[bad[:8]]} want {want[bad[:8]]}"
    if policy == 1:  # the reference pool's metric units
        assert (st.batch_retries, st.batch_sigs_success) == (ost.batch_retries, ost.batch_sigs_success)
    return got, st


def test_c5_mixed_vs_oracle(ctx):
    w, n, desc, _ = bench.build_workload(ctx, "C5", 0, signer=oracle_sign)
    assert desc["invalid_sets"] == 10 and n == 1024
    table = bench.oracle_table(w)
    got, st = compare(ctx, call_of(w), table)
    assert np.array_equal(got, w["expected"]) and st.batch_retries >= 1
    compare(ctx, call_of(w), table, policy=1)
    compare(ctx, call_of(w), table, seed=12345)
    compare(ctx, call_of(w, job_flags=np.zeros(len(w["expected"]), np.uint8)), table)  # every job its own group
    bad, applied = corrupted(w, 0xC5)
    got, _ = compare(ctx, bad, table)
    assert len(set(got.tolist())) >= 5
    compare(ctx, bad, table, policy=1)


def test_c3_block_import_vs_oracle(ctx):
    w, n, desc, k = bench.build_workload(ctx, "C3", 0, signer=oracle_sign)
    assert n == 128 and k == 512
    table = bench.oracle_table(w)
    got, _ = compare(ctx, call_of(w), table)
    assert list(got) == [1]
    # as 128 separate batchable jobs, then with one pubkey index of set 77 swapped (only job 77 false)
    jfs = np.arange(n + 1, dtype=np.uint32)
    got, _ = compare(ctx, call_of(w, job_first_set=jfs, job_flags=np.ones(n, np.uint8)), table)
    assert (got == 1).all()
    pk = w["pk_index"].copy()
    pk[77 * 512 + 5] = 65535 - pk[77 * 512 + 5]
    got, _ = compare(ctx, call_of(w, job_first_set=jfs, job_flags=np.ones(n, np.uint8), pk_index=pk), table)
    want = np.ones(n, np.int8)
    want[77] = 0
    assert np.array_equal(got, want)
    bad, _ = corrupted(w, 0xC3)
    compare(ctx, dict(bad, job_first_set=jfs, job_flags=np.ones(n, np.uint8)), table)
    compare(ctx, dict(bad, job_first_set=jfs, job_flags=np.ones(n, np.uint8)), table, policy=1)


@pytest.mark.parametrize("world", [8, 1])
def test_c4_epoch_vs_oracle(ctx, world):
    """world 8: one rank's shard (4,096 aggregate sets); world 1: the whole 32,768-set step on one device.  The
    pubkeys come from the 2^20-validator device table."""
    w, n, desc, _ = bench.build_workload(ctx, "C4", 0, world, signer=oracle_sign)
    assert n == 32768 // world and desc["total_sets_per_step"] == 32768
    assert ctx.pubkeys_count >= 1 << 20
    table = bench.oracle_table(w)
    got, st = compare(ctx, call_of(w), table)
    assert (got == 1).all() and st.batch_retries == 0
    if world == 8:
        sigs = w["sigs"].copy()
        sigs[96 * 1000: 96 * 1001] = w["sigs"][96 * 1001: 96 * 1002]  # set 1001's sig on set 1000 (same committee)
        got, _ = compare(ctx, call_of(w, sigs=sigs), table)
        assert list(np.nonzero(got != 1)[0]) == [1000] and got[1000] == 0
        bad, _ = corrupted(w, 0xC4)
        compare(ctx, bad, table)
        compare(ctx, bad, table, policy=1)


def test_pool_policy_split_calls_vs_oracle(ctx):
    """group_policy 1 on calls that the pool splits (> 128 sets: chunkify(sets, 128)) mixed with small batchable and
    non-batchable calls and an empty call: per-call answers and the pool's metric units equal the oracle's."""
    rng = np.random.default_rng(77)
    sizes = [300, 1, 2, 129, 0, 64, 1, 1, 513, 7, 3, 128, 1, 40]
    flags = [1, 1, 0, 1, 1, 0, 1, 0, 1, 1, 1, 0, 1, 1]
    n = sum(sizes)
    sks = [bench.interop_sk(i).to_bytes(32, "big") for i in range(n)]
    msgs = [bench.msg_j(j, 0x9001) for j in range(n)]
    sigs = oracle_sign(b"".join(sks), b"".join(msgs))
    pks = cpu.sk_to_pk(b"".join(sks), threads=THREADS)
    m2, buf, sl, _ = corrupt.corrupt_sets([sigs[96 * i: 96 * i + 96] for i in range(n)], msgs, rng, frac=0.004)
    call = dict(job_first_set=np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint32), sigs=buf, sig_len=sl,
                msgs=b"".join(m2), pk_bytes=pks, job_flags=np.asarray(flags, np.uint8), sig_stride=192)
    got, st = compare(ctx, call, None, policy=1)
    assert got[4] == -10  # the empty call: "Empty signature set"
    compare(ctx, call, None, policy=0)
    clean = dict(call, sigs=sigs, sig_len=[96] * n, msgs=b"".join(msgs), sig_stride=96)
    got, st = compare(ctx, clean, None, policy=1)
    assert (np.delete(got, 4) == 1).all() and st.batch_retries == 0


def test_c5_lane_tails_vs_oracle(ctx):
    """The lane forms of the signature tails (two-lane Horner passes, one-lane MillerLoop(-g1, S) per group; merged
    runs by default) forced on every run of the C5 workload: the same results as the oracle job for job."""
    w, n, desc, _ = bench.build_workload(ctx, "C5", 0, signer=oracle_sign)
    table = bench.oracle_table(w)
    ctx.set_option("lane_tail_min", 1)
    try:
        got, st = compare(ctx, call_of(w), table)
    finally:
        ctx.set_option("lane_tail_min", 0)
    assert np.array_equal(got, w["expected"])


@pytest.mark.parametrize("opts", [
    {"fb_force_busy": 1, "fb_direct_min": 1, "fb_lane_min": 1},                  # every job: six-lane Miller + gt6
    {"fb_force_busy": 1, "fb_direct_min": 0, "fb_lane_min": 1, "small_max": 0},  # sub-groups, then jobs
    {"fb_force_busy": 1, "fb_direct_min": 1, "fb_lane_min": 1, "fb_check6": 1},  # one-lane Miller + gt6
])
def test_c5_under_load_fallback_forms_vs_oracle(ctx, opts):
    """C5's fallback in the forms merged runs take under load (six-lane, or one-lane, MillerLoop(-g1, S) and the six-lane final
    exponentiation of gt6.hpp per check; per job directly or after sub-groups), forced on a lone call: job for job equal
    to the oracle, on the reference-shaped workload and on a copy with every corruption class."""
    w, n, desc, _ = bench.build_workload(ctx, "C5", 0, signer=oracle_sign)
    table = bench.oracle_table(w)
    saved = {k: ctx.get_option(k) for k in opts}
    try:
        for k, v in opts.items():
            ctx.set_option(k, v)
        got, st = compare(ctx, call_of(w), table)
        assert np.array_equal(got, w["expected"]) and st.fallback_jobs > 0
        bad, _ = corrupted(w, 0xC6)
        compare(ctx, bad, table)
    finally:
        for k, v in saved.items():
            ctx.set_option(k, v)

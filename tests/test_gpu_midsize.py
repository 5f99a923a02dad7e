"""GPU parity of mid-size calls (1k-8k sets: gossip batches, sync-batch chunks -- reference multithread/index.ts:34,39,
worker.ts:17,56) job for job against the C restatement of the reference pool (oracle/blscpu.c verify_jobs), with ~1%
of the sets corrupted in every way the reference distinguishes (oracle/corrupt.py), jobs of 1-3 sets.  Covers the
forms a run of this size can take: the cooperative Miller loops and [|z|] chains (runtime options coop_max /
coop_g2_max), the lane forms, the speculative r_i sig_i of small idle runs (rsig_spec) and the fallback that reuses
the batch pass's per-set Miller values (blsgpu_stats.fallback_miller == 0) or, with same-message units, recomputes
them."""
import numpy as np
import pytest

import bench
from oracle import corrupt, cpu

pytestmark = pytest.mark.gpu

THREADS = bench.host_cpus()["threads"]
N_MAX = 8192


@pytest.fixture(scope="module")
def ctx():
    from lodestar_amd.native import Context

    c = Context([0])
    yield c
    c.close()


@pytest.fixture(scope="module")
def pool():
    """N_MAX oracle-signed single-key sets over distinct roots, their keys in bytes form."""
    sks = [bench.interop_sk(i).to_bytes(32, "big") for i in range(N_MAX)]
    msgs = [bench.msg_j(j, 0x3151) for j in range(N_MAX)]
    sigs = cpu.sign(b"".join(sks), b"".join(msgs), threads=THREADS)
    pks = cpu.sk_to_pk(b"".join(sks), threads=THREADS)
    return sks, msgs, sigs, pks


def job_split(n, seed):
    rng = np.random.default_rng(seed)
    sizes, left = [], n
    while left:
        k = min(left, int(rng.integers(1, 4)))
        sizes.append(k)
        left -= k
    return np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint32)


def make_call(pool, n, seed, frac=0.01, share_every=0):
    sks, msgs, sigs, pks = pool
    m = list(msgs[:n])
    s = [sigs[96 * i: 96 * i + 96] for i in range(n)]
    if share_every:  # groups of sets signing one root (same-message pairing units): re-sign them
        for i in range(n):
            m[i] = msgs[(i // share_every) * share_every]
        s = cpu.sign(b"".join(sks[:n]), b"".join(m), threads=THREADS)
        s = [s[96 * i: 96 * i + 96] for i in range(n)]
    m2, buf, sl, applied = corrupt.corrupt_sets(s, m, np.random.default_rng(seed), frac=frac)
    jfs = job_split(n, seed)
    return dict(job_first_set=jfs, sigs=buf, sig_len=sl, msgs=b"".join(m2), pk_bytes=pks[: 96 * n],
                job_flags=np.ones(len(jfs) - 1, np.uint8), sig_stride=192), applied


def compare(ctx, call, seed=bench.SEED):
    got, st = ctx.verify_raw(**call, seed=seed)
    want, _ = cpu.verify_jobs(table=None, threads=THREADS, **call, seed=seed)
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, f"{len(bad)} mismatches, first {bad[:8]}: got {got[bad[:8]]} want {want[bad[:8]]}"
    return got, st


@pytest.mark.parametrize("n", [512, 513, 1024, 2048, 4096, 8192])
def test_midsize_one_percent_corrupt_vs_oracle(ctx, pool, n):
    """The verdict's mid-size parity: 1k / 2k / 4k / 8k sets, ~1% corrupted, at the runtime defaults (up to 512
    pairings the cooperative Miller loops -- 512 / 513 sit on either side of that edge --, up to 4k the cooperative
    chains, 8k the lane forms); the failed groups' per-job checks reuse the batch pass's Miller values."""
    call, applied = make_call(pool, n, 0x5000 + n)
    assert len(applied) >= n // 200
    got, st = compare(ctx, call)
    assert (got == 1).sum() > len(got) // 2 and (got != 1).sum() >= 1
    assert st.fallback_jobs > 0 and st.fallback_miller == 0


@pytest.mark.parametrize("opts", [
    {"coop_max": 0, "coop_g2_max": 0},              # lane forms at 1k
    {"coop_max": 1 << 20, "coop_g2_max": 1 << 20},  # cooperative forms everywhere
    {"rsig_spec": 0},                               # the fallback forms r_i sig_i itself
    {"coop_excl_max": 1 << 20},                     # exclusive CUs for every cooperative launch
    {"fb_lane_min": 1, "coop_max": 0},              # lane-per-check fallback checks (merged runs under load)
    {"coop_max": 0, "acc6_max": 0},                 # two-lane accumulation instead of the six-lane one
    {"coop_max": 0, "miller_lanes": 6, "dedupe": 0},  # six lanes forced
    {"coop_max": 0, "miller_lanes": 3},               # lane pairs (gtx.hpp) for the batch pass and the fallback
    # the fallback's under-load forms: one-lane MillerLoop(-g1, S) + six-lane final exponentiations (gt6.hpp), per job
    # directly or after sub-groups; and the all-one-lane checks
    {"fb_force_busy": 1, "fb_direct_min": 1, "fb_lane_min": 1},
    {"fb_force_busy": 1, "fb_direct_min": 0, "fb_lane_min": 1, "small_max": 0},
    {"fb_force_busy": 1, "fb_direct_min": 1, "fb_lane_min": 1, "fb_check6": 0},
    {"fb_force_busy": 1, "fb_direct_min": 1, "fb_lane_min": 1, "fb_check6": 1},
])
def test_midsize_forms_agree(ctx, pool, opts):
    saved = {k: ctx.get_option(k) for k in opts}
    try:
        for k, v in opts.items():
            ctx.set_option(k, v)
        for n in (1024, 3000):
            call, _ = make_call(pool, n, 0x6000 + n)
            compare(ctx, call)
    finally:
        for k, v in saved.items():
            ctx.set_option(k, v)


@pytest.mark.parametrize("lanes", [0, 3])
def test_fallback_units_recompute_vs_oracle(ctx, pool, lanes):
    """Same-message units (4 sets per root): the batch pass pairs units, not sets, so the fallback recomputes the
    failed jobs' Miller loops (fallback_miller > 0) -- still job for job equal to the oracle (default Miller forms, and
    lane pairs for every accumulation)."""
    call, _ = make_call(pool, 2048, 0x7000, share_every=4)
    saved = (ctx.get_option("miller_lanes"), ctx.get_option("coop_max"))
    ctx.set_option("miller_lanes", lanes)
    if lanes:
        ctx.set_option("coop_max", 0)
    try:
        got, st = compare(ctx, call)
    finally:
        ctx.set_option("miller_lanes", saved[0])
        ctx.set_option("coop_max", saved[1])
    assert st.fallback_jobs > 0 and st.fallback_miller > 0


def test_midsize_all_valid_no_fallback(ctx, pool):
    sks, msgs, sigs, pks = pool
    n = 4096
    jfs = job_split(n, 9)
    call = dict(job_first_set=jfs, sigs=sigs[: 96 * n], sig_len=np.full(n, 96, np.uint32), msgs=b"".join(msgs[:n]),
                pk_bytes=pks[: 96 * n], job_flags=np.ones(len(jfs) - 1, np.uint8), sig_stride=96)
    got, st = ctx.verify_raw(**call)
    assert (got == 1).all() and st.fallback_jobs == 0 and st.batch_retries == 0


def test_mainnet_g2_corpus_in_pipeline(ctx, pool):
    """All 55 reference-held mainnet G2 encodings (tests/golden/mainnet_g2_points.json: blocks.json's 53 + the
    aggregator.test.ts proofs) as the signatures of single-set jobs over other keys and roots: every one decodes and
    passes the subgroup check inside the verification pipeline (result 0 = well-formed, wrong equation, never an
    error code), in the cooperative and the lane forms of the subgroup check, as the oracle says."""
    import json
    import os

    sks, msgs, sigs, pks = pool
    pts = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "mainnet_g2_points.json")))["points"]
    n = len(pts)
    assert n >= 55
    call = dict(job_first_set=np.arange(n + 1, dtype=np.uint32), sigs=b"".join(bytes.fromhex(h) for h in pts),
                sig_len=np.full(n, 96, np.uint32), msgs=b"".join(msgs[:n]), pk_bytes=pks[: 96 * n],
                job_flags=np.ones(n, np.uint8), sig_stride=96)
    saved = ctx.get_option("coop_g2_max")
    try:
        for g2 in (1 << 20, 0):
            ctx.set_option("coop_g2_max", g2)
            got, _ = compare(ctx, call)
            assert (got == 0).all()
    finally:
        ctx.set_option("coop_g2_max", saved)


def test_routing_whole_calls_and_split_epoch_calls(pool):
    """Calls are routed, not sharded (runtime route_rule): on two device contexts a 16k gossip call runs whole on one
    device, a 32,768-set call (C4's step) splits over both, and concurrent whole calls spread over the devices."""
    from concurrent.futures import ThreadPoolExecutor

    from lodestar_amd.native import Context

    sks, msgs, sigs, pks = pool
    c2 = Context([0, 0])
    try:
        for reps, want_dev in ((2, 1), (4, 2)):
            n = N_MAX * reps
            call = dict(job_first_set=np.arange(n + 1, dtype=np.uint32), sigs=sigs * reps,
                        sig_len=np.full(n, 96, np.uint32), msgs=b"".join(msgs) * reps, pk_bytes=pks * reps,
                        job_flags=np.ones(n, np.uint8), sig_stride=96)
            got, st = c2.verify_raw(**call)
            assert (got == 1).all() and st.devices_used == want_dev, (n, st.devices_used)
        n = 2048
        call = dict(job_first_set=np.arange(n + 1, dtype=np.uint32), sigs=sigs[: 96 * n],
                    sig_len=np.full(n, 96, np.uint32), msgs=b"".join(msgs[:n]), pk_bytes=pks[: 96 * n],
                    job_flags=np.ones(n, np.uint8), sig_stride=96)
        with ThreadPoolExecutor(4) as ex:
            outs = list(ex.map(lambda _: c2.verify_raw(**call), range(8)))
        assert all((g == 1).all() and st.devices_used == 1 for g, st in outs)
    finally:
        c2.close()


def test_large_failing_jobs_fallback_vs_oracle(ctx, pool):
    """Advisor r5: retried jobs of ~1k sets each in a small idle run (r_i sig_i formed speculatively) take the bucket
    MSM and the wave-per-job reduce, not the one-lane reduce over thousands of sets.  Three 1,024-set block-shaped jobs
    in one batch group (group_sets 4096), two of them with one set signed over another root, then 64 one-set jobs:
    job for job equal to the oracle; the fallback re-checks the group's clean jobs."""
    import time

    sks, msgs, sigs, pks = pool
    n = 3 * 1024 + 64
    m = list(msgs[:n])
    for bad in (100, 1024 + 700):  # jobs 0 and 1: one set over another root
        m[bad] = msgs[N_MAX - 1 - bad]
    sizes = [1024, 1024, 1024] + [1] * 64
    call = dict(job_first_set=np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint32), sigs=sigs[: 96 * n],
                sig_len=np.full(n, 96, np.uint32), msgs=b"".join(m), pk_bytes=pks[: 96 * n],
                job_flags=np.ones(len(sizes), np.uint8), sig_stride=96)
    saved = ctx.get_option("group_sets")
    ctx.set_option("group_sets", 4096)
    try:
        t0 = time.perf_counter()
        got, st = compare(ctx, call)
        print(f"two failing 1k-set jobs: {1e3 * (time.perf_counter() - t0):.1f} ms, fallback_jobs {st.fallback_jobs}")
    finally:
        ctx.set_option("group_sets", saved)
    assert list(got[:3]) == [0, 0, 1] and (got[3:] == 1).all()
    assert st.fallback_jobs >= 3

"""GPU parity at BASELINE.json's config sizes through size-independent properties (the CPU oracle is far too
slow for 10^4 pairings): every valid set verifies, every set signed over the wrong message makes exactly its
own job false (invalid-batch fallback), results do not depend on batching or on the random scalars, and a
corrupted aggregate fails only its own job.  Workloads come from bench.py's generators."""
import numpy as np
import pytest

import bench

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from lodestar_amd.native import Context

    c = Context([0])
    yield c
    c.close()


def run(ctx, w, seed=bench.SEED, **over):
    call = {k: v for k, v in w.items() if k not in ("expected", "pks_table") and not k.startswith("_")}
    call.update(over)
    res, st = ctx.verify_raw(**call, seed=seed)
    return res, st


def test_c5_mixed_one_percent_invalid(ctx):
    w, n, desc, _ = bench.build_workload(ctx, "C5", 0)
    assert desc["invalid_sets"] == 10
    res, st = run(ctx, w)
    assert np.array_equal(res, w["expected"])
    assert st.batch_retries >= 1  # the failing groups went through the fallback
    # independent of the batch scalars and of batching (non-batchable: each job its own group)
    res2, _ = run(ctx, w, seed=12345)
    assert np.array_equal(res2, w["expected"])
    res3, _ = run(ctx, w, job_flags=np.zeros(len(w["expected"]), np.uint8))
    assert np.array_equal(res3, w["expected"])
    # a message variant of the bench's in-flight pool (new roots, re-signed): the same per-job answers
    w1 = bench.message_variant(ctx, w, 3)
    assert not np.array_equal(w1["msgs"], w["msgs"])
    res4, _ = run(ctx, w1)
    assert np.array_equal(res4, w["expected"])


def test_c3_block_import_aggregates(ctx):
    w, n, desc, k = bench.build_workload(ctx, "C3", 0)
    assert n == 128 and k == 512
    res, _ = run(ctx, w)
    assert list(res) == [1]
    # as 128 separate jobs, then with one pubkey index of set 77 swapped (wrong aggregate -> only job 77 false)
    jfs = np.arange(n + 1, dtype=np.uint32)
    res, _ = run(ctx, w, job_first_set=jfs, job_flags=np.ones(n, np.uint8))
    assert (res == 1).all()
    pk = w["pk_index"].copy()
    pk[77 * 512 + 5] = 65535 - pk[77 * 512 + 5]
    res, _ = run(ctx, w, job_first_set=jfs, job_flags=np.ones(n, np.uint8), pk_index=pk)
    want = np.ones(n, np.int8)
    want[77] = 0
    assert np.array_equal(res, want)


def test_c4_shard_of_epoch(ctx):
    """One rank's shard of C4 (world 8): 4,096 aggregate sets over the 2^20-validator table."""
    w, n, desc, _ = bench.build_workload(ctx, "C4", 0, 8)
    assert n == 4096 and desc["total_sets_per_step"] == 32768
    assert ctx.pubkeys_count >= 1 << 20
    res, st = run(ctx, w)
    assert (res == 1).all() and st.batch_retries == 0
    sigs = w["sigs"].copy()
    sigs[96 * 1000 : 96 * 1001] = w["sigs"][96 * 1001 : 96 * 1002]  # set 1001's sig on set 1000 (same committee)
    res, _ = run(ctx, w, sigs=sigs)
    assert list(np.nonzero(res != 1)[0]) == [1000] and res[1000] == 0

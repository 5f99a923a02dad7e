"""C5 under load, many calls: bench.py's C5 workload (1,024 sets in jobs of 1-3, 1% signed over another message) with
every call's message variant re-signed on the device, 32 calls in flight for ROUNDS rounds (the bench's warm-up
shape), each call's per-job verdicts checked
against the expected ones, and no batch group may fail while all its jobs verify alone (the runtime's
"spurious_groups" count).  A mismatch is diagnosed before the test fails: the same call re-verified alone on the GPU,
and the job's sets through the CPU oracle (oracle/blscpu.c) -- which separates a wrong device-made signature (both
agree with each other), a transient verifier error (the lone call is right) and a persistent one.  The details go
to gpurun_out/c5_stress_fail.json."""
import json
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import bench
from oracle import cpu

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
THREADS = bench.host_cpus()["threads"]
ROUNDS = int(os.environ.get("C5_STRESS_ROUNDS", "48"))
# one message variant per call in flight (+1), as bench.py: merged runs share no signing root, so the runs keep their
# per-set Miller values for the fallback (runtime keep_f) -- with fewer variants merged calls share roots and pair by
# units instead
VARIANTS = int(os.environ.get("C5_STRESS_VARIANTS", "33"))


@pytest.fixture(scope="module")
def env():
    from lodestar_amd.native import Context

    ctx = Context([0])
    w, n, desc, _ = bench.build_workload(ctx, "C5", 0)
    expected = w.pop("expected")
    strip = lambda x: {k: v for k, v in x.items() if not k.startswith("_")}
    calls = [strip(bench.message_variant(ctx, w, v)) for v in range(VARIANTS)]
    yield ctx, w, calls, expected
    ctx.close()


def diagnose(ctx, w, call, expected, got, st, v):
    bad = np.nonzero(got != expected)[0]
    alone, _ = ctx.verify_raw(**call, seed=bench.SEED)
    jfs = call["job_first_set"]
    rows = []
    table = cpu.Table(w["_table_pks"])
    for j in bad[:8].tolist():
        s0, s1 = int(jfs[j]), int(jfs[j + 1])
        spf = call["set_pk_first"]
        sub = dict(job_first_set=np.array([0, s1 - s0], np.uint32), sigs=call["sigs"][96 * s0: 96 * s1],
                   sig_len=call["sig_len"][s0:s1], msgs=call["msgs"][32 * s0: 32 * s1],
                   set_pk_first=(spf[s0: s1 + 1] - spf[s0]).astype(np.uint32),
                   pk_index=call["pk_index"][spf[s0]: spf[s1]], job_flags=call["job_flags"][j: j + 1], sig_stride=96)
        want, _ = cpu.verify_jobs(table=table, threads=THREADS, **sub, seed=bench.SEED)
        gpu_sub, _ = ctx.verify_raw(**sub, seed=bench.SEED)
        rows.append({"job": j, "sets": [s0, s1], "got": int(got[j]), "expected": int(expected[j]),
                     "alone_gpu": int(alone[j]), "oracle_job": int(want[0]), "gpu_job_alone": int(gpu_sub[0])})
    return {"variant": v, "mismatched_jobs": bad.tolist(), "stats": {k: getattr(st, k) for k, _ in st._fields_},
            "jobs": rows}


# fixed and adaptive groups (option group_adapt, DESIGN.md 5.2: with outgrown buffers returned to the pool at once the
# adaptive groups answered false for valid jobs in ~6% of fresh bench processes, never inside this test's one process)
@pytest.mark.parametrize("adapt", [0, 1])
def test_c5_many_calls_under_load(env, adapt):
    """ROUNDS rounds of 32 calls in flight (the calls of a round cycle through the variants)."""
    ctx, w, calls, expected = env
    old = ctx.get_option("group_adapt")
    ctx.set_option("group_adapt", adapt)
    failures = []

    def step(i):
        v = i % VARIANTS
        got, st = ctx.verify_raw(**calls[v], seed=bench.SEED)
        if not np.array_equal(got, expected):
            return (i, v, got, st)
        return None

    try:
        with ThreadPoolExecutor(max_workers=32) as pool:
            for r in range(ROUNDS):
                for res in pool.map(step, range(r * 32, (r + 1) * 32)):
                    if res is not None:
                        failures.append(res)
                if failures:
                    break
    finally:
        ctx.set_option("group_adapt", old)
    spurious = ctx.get_option("spurious_groups")
    if failures:
        i, v, got, st = failures[0]
        info = diagnose(ctx, w, calls[v], expected, got, st, v)
        info.update(call=i, adapt=adapt, failures=len(failures))
        os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
        with open(os.path.join(ROOT, "gpurun_out", "c5_stress_fail.json"), "w") as fh:
            json.dump(info, fh, indent=1, default=str)
        pytest.fail(f"C5 mismatch: {json.dumps(info, default=str)[:2000]}")
    assert spurious == 0, f"{spurious} batch groups failed although all their jobs verify (see stderr)"


COLD = int(os.environ.get("C5_COLD_ROUNDS", "4"))


def test_c5_cold_contexts():
    """The bench's cold start, COLD times: a fresh context, the C5 workload and its message variants signed on the
    device, one round of 32 calls in flight.  On a mismatch the job's sets go through the CPU oracle with the
    device-made signatures: oracle false = the device SIGNER made a wrong signature (a test-input fault, not a
    verifier one); oracle true = the verifier answered wrong."""
    from lodestar_amd.native import Context

    strip = lambda x: {k: v for k, v in x.items() if not k.startswith("_")}
    for it in range(COLD):
        ctx = Context([0])
        try:
            w, n, desc, _ = bench.build_workload(ctx, "C5", 0)
            expected = w.pop("expected")
            calls = [strip(bench.message_variant(ctx, w, v)) for v in range(32)]
            with ThreadPoolExecutor(max_workers=32) as pool:
                res = list(pool.map(lambda v: ctx.verify_raw(**calls[v], seed=bench.SEED), range(32)))
            for v, (got, st) in enumerate(res):
                if not np.array_equal(got, expected):
                    info = diagnose(ctx, w, calls[v], expected, got, st, v)
                    info.update(cold_iteration=it)
                    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
                    with open(os.path.join(ROOT, "gpurun_out", "c5_cold_fail.json"), "w") as fh:
                        json.dump(info, fh, indent=1, default=str)
                    signer = all(r["oracle_job"] == r["got"] for r in info["jobs"])
                    pytest.fail(("device SIGNER fault" if signer else "VERIFIER fault") +
                                f": {json.dumps(info, default=str)[:2000]}")
            assert ctx.get_option("spurious_groups") == 0
        finally:
            ctx.close()

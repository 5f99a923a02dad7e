"""The urgent lane (BLSGPU_JOB_URGENT, the reference's VerifySignatureOpts.verifyOnMainThread): a latency-critical call
-- the gossip block proposer signature (reference chain/validation/block.ts:146), which the reference verifies at once on
the main thread, outside the pool queue (multithread/index.ts:138-151) -- submitted behind a gossip flood of 16,384-set
calls completes before the flood does, with the oracle's answer: valid, a signature over the wrong message, a malformed
signature, and 3-set calls.  Results are compared job for job with oracle/blscpu.c on the same inputs and seed."""
import threading
import time

import numpy as np
import pytest

import bench
from lodestar_amd.native import JOB_BATCHABLE, JOB_URGENT
from oracle import cpu

pytestmark = pytest.mark.gpu

THREADS = bench.host_cpus()["threads"]
N_FLOOD, FLOOD_CALLS, N_KEYS = 16384, 16, 16384


@pytest.fixture(scope="module")
def env():
    from lodestar_amd.native import Context

    ctx = Context([0])
    sks = [bench.interop_sk(i).to_bytes(32, "big") for i in range(N_KEYS)]
    pks = cpu.sk_to_pk(b"".join(sks), threads=THREADS)
    ctx.upload_pubkeys(0, pks)
    # the flood: FLOOD_CALLS gossip calls of 16,384 batchable single sets over distinct roots (signed on the GPU: they
    # only load the device, their results are checked to be all valid)
    flood = []
    for c in range(FLOOD_CALLS):
        msgs = [bench.msg_j(c * N_FLOOD + j, 0x4F4C46) for j in range(N_FLOOD)]
        sigs = bench.gen_sigs(ctx, sks[:N_FLOOD], msgs)
        flood.append(dict(job_first_set=np.arange(N_FLOOD + 1, dtype=np.uint32), sigs=np.frombuffer(sigs, np.uint8),
                          sig_len=np.full(N_FLOOD, 96, np.uint32), msgs=np.frombuffer(b"".join(msgs), np.uint8),
                          set_pk_first=np.arange(N_FLOOD + 1, dtype=np.uint32),
                          pk_index=np.arange(N_FLOOD, dtype=np.uint32),
                          job_flags=np.full(N_FLOOD, JOB_BATCHABLE, np.uint8), sig_stride=96))
    yield ctx, sks, pks, flood
    ctx.close()


def urgent_call(sks, idx, kinds, seed_tag):
    """One urgent job over the sets `idx` (table mode), oracle-signed; kinds[i]: 'ok', 'wrong_msg' (signed over another
    root -> false), 'bad_encoding' (compression flag cleared -> BLST_BAD_ENCODING)."""
    msgs = [bench.msg_j(7_000_000 + seed_tag * 8 + i, 0x55524745) for i in range(len(idx))]
    signed = [bench.msg_j(9_000_000 + seed_tag * 8 + i, 0x55524745) if k == "wrong_msg" else m
              for i, (m, k) in enumerate(zip(msgs, kinds))]
    sigs = bytearray(cpu.sign(b"".join(sks[i] for i in idx), b"".join(signed), threads=THREADS))
    for i, k in enumerate(kinds):
        if k == "bad_encoding":
            sigs[96 * i] &= 0x7F
    n = len(idx)
    return dict(job_first_set=np.array([0, n], np.uint32), sigs=np.frombuffer(bytes(sigs), np.uint8),
                sig_len=np.full(n, 96, np.uint32), msgs=np.frombuffer(b"".join(msgs), np.uint8),
                set_pk_first=np.arange(n + 1, dtype=np.uint32), pk_index=np.array(idx, np.uint32),
                job_flags=np.array([JOB_URGENT], np.uint8), sig_stride=96)


URGENT_CASES = [
    ([11], ["ok"], 1),
    ([12], ["wrong_msg"], 0),
    ([13], ["bad_encoding"], -1),
    ([21, 22, 23], ["ok", "ok", "ok"], 1),
    ([31, 32, 33], ["ok", "wrong_msg", "ok"], 0),
]


def oracle_result(pks, call, seed):
    want, _ = cpu.verify_jobs(table=cpu.Table(pks), threads=THREADS, **call, seed=seed)
    return int(want[0])


def test_urgent_calls_alone_vs_oracle(env):
    """Urgent calls on an idle device: the lane's answer is the oracle's, and the stats say the lane ran them."""
    ctx, sks, pks, _ = env
    for t, (idx, kinds, expect) in enumerate(URGENT_CASES):
        call = urgent_call(sks, idx, kinds, t)
        got, st = ctx.verify_raw(**call, seed=bench.SEED + t)
        want = oracle_result(pks, call, bench.SEED + t)
        assert int(got[0]) == want, (kinds, got, want)
        assert (want == expect) if expect >= 0 else want < 0
        assert st.urgent_lane == 1


def run_behind_flood(ctx, flood, calls, seeds, twin=None):
    """Queues the flood (FLOOD_CALLS threads), then after 30 ms submits the urgent calls together (and, with `twin`, the
    same calls without the urgent flag, as ordinary calls queued behind the flood).  Returns (urgent outcomes [(result,
    lane, ms, done_t)], twin outcomes, sorted flood completion times (ms from the flood's submission))."""
    done, errs = [None] * FLOOD_CALLS, []

    def flood_call(k):
        try:
            res, _ = ctx.verify_raw(**flood[k], seed=bench.SEED)
            if not (res == 1).all():
                errs.append(f"flood call {k}: {(res != 1).sum()} jobs not valid")
        except Exception as e:  # noqa: BLE001 -- reported below
            errs.append(repr(e))
        done[k] = time.perf_counter()

    def one(c, seed, out, t):
        t1 = time.perf_counter()
        got, st = ctx.verify_raw(**c, seed=seed)
        out[t] = (int(got[0]), int(st.urgent_lane), (time.perf_counter() - t1) * 1e3, time.perf_counter())

    th = [threading.Thread(target=flood_call, args=(k,)) for k in range(FLOOD_CALLS)]
    t0 = time.perf_counter()
    for x in th:
        x.start()
    time.sleep(0.03)  # the flood is queued on the device
    outs, touts = [None] * len(calls), [None] * len(calls)
    uth = [threading.Thread(target=one, args=(c, seeds[t], outs, t)) for t, c in enumerate(calls)]
    if twin:
        uth += [threading.Thread(target=one, args=(dict(c, job_flags=np.zeros(1, np.uint8)), seeds[t], touts, t))
                for t, c in enumerate(calls)]
    for x in uth:
        x.start()
    for x in uth + th:
        x.join(timeout=120)
    assert not errs, errs
    rel = lambda o: [(r, lane, ms, (d - t0) * 1e3) for r, lane, ms, d in o] if o[0] else None
    return rel(outs), rel(touts) if twin else None, sorted((d - t0) * 1e3 for d in done)


def test_urgent_calls_overtake_a_gossip_flood(env):
    """FLOOD_CALLS x 16,384-set calls (two merged pipeline runs of 131,072 sets) are queued first, then the urgent calls
    (valid, wrong message, malformed signature, 3-set jobs) and the same calls without the urgent flag, submitted
    together: every urgent call gives the oracle's answer on the urgent lane (the burst merged into one lane run), and
    all of them finish before the ordinary copies, which wait behind the flood in the device queue.  (With an isolated CU
    partition, `urgent_cus` 8, they also finish before the flood's median call: measured by bench.py in processes of
    their own, profiles/r06_urgent_latency.json -- a second context with CU-masked pipeline streams beside this one
    exhausted the scratch the extra hardware queues reserve)"""
    ctx, sks, pks, flood = env
    calls = [urgent_call(sks, idx, kinds, 100 + t) for t, (idx, kinds, _) in enumerate(URGENT_CASES)]
    seeds = [bench.SEED + 100 + t for t in range(len(calls))]
    wants = [oracle_result(pks, c, s) for c, s in zip(calls, seeds)]
    ctx.verify_raw(**calls[0], seed=seeds[0])  # the lane's buffers exist before timing
    outs, touts, flood_ms = run_behind_flood(ctx, flood, calls, seeds, twin=True)
    u_done = max(o[3] for o in outs)
    t_done = min(o[3] for o in touts)
    print(f"urgent latencies behind the flood (ms): {[round(o[2], 2) for o in outs]}, done at {u_done:.1f} ms; flood "
          f"done at {flood_ms[0]:.1f} .. {flood_ms[-1]:.1f} ms; the same calls queued as ordinary calls done at "
          f"{t_done:.1f} .. {max(o[3] for o in touts):.1f} ms")
    for t, o in enumerate(outs):
        assert o[0] == wants[t], (t, o, wants[t])
        assert o[1] == 1
    for t, o in enumerate(touts):
        assert o[0] == wants[t] and o[1] == 0
    assert u_done < t_done, "urgent calls did not overtake the queue"


def test_large_urgent_call_takes_the_queue_head(env):
    """An urgent call above urgent_max_sets runs on the pipeline (queued at the head of the device queue), with the
    oracle's answer; with the lane off an urgent call is an ordinary call."""
    ctx, sks, pks, _ = env
    old_max, old_lane = ctx.get_option("urgent_max_sets"), ctx.get_option("urgent_lane")
    try:
        ctx.set_option("urgent_max_sets", 2)
        call = urgent_call(sks, [41, 42, 43], ["ok", "ok", "wrong_msg"], 200)
        got, st = ctx.verify_raw(**call, seed=bench.SEED)
        assert int(got[0]) == oracle_result(pks, call, bench.SEED) == 0
        assert st.urgent_lane == 0
        ctx.set_option("urgent_max_sets", old_max)
        ctx.set_option("urgent_lane", 0)
        call = urgent_call(sks, [44], ["ok"], 201)
        got, st = ctx.verify_raw(**call, seed=bench.SEED)
        assert int(got[0]) == 1 and st.urgent_lane == 0
    finally:
        ctx.set_option("urgent_max_sets", old_max)
        ctx.set_option("urgent_lane", old_lane)

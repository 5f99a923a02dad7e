"""GPU tests of the failure paths: the speculative small-run MSM's exactness, fail-closed batch scalars, injected
device failures, and the in-process two-shard path at C4's full size.

* Speculative MSM (runtime.cpp run_shard, `spec`): an idle small run sums every DECODED signature into S_g before
  the job mask exists, so a group holding a rejected job (a signature outside G2, a bad pubkey) is not the equation
  of its clean jobs; those must be re-checked with exact masks.  Cases: a 2-job call with one such job and one valid
  job -> [-code, 1] (the advisor's counterexample), and an idle 128-set call mixing a non-G2 signature, a
  wrong-message set and valid sets, job for job against the oracle (oracle/blscpu.c verify_jobs).
* Batch scalars: seed 0 (production) verifies like the oracle; an entropy failure refuses the call
  (BLSGPU_ERR_ENTROPY, every job rejected), never a constant fallback.
* Device failure (reference multithread/index.ts:368-375): an injected HIP failure rejects every job of
  every call in the failing run with -BLSGPU_DEVICE_ERROR (never 0), including calls merged into that run, and the
  dispatcher keeps serving: the next calls verify.
* Context([0, 0]) on C4's 32,768 aggregate sets over the 2^20-key table: both shards' tables filled by the
  concurrent upload, results job for job equal to the oracle.
"""
import threading
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import bench
from oracle import bls12_381 as bls
from oracle import corrupt, cpu
from tests.test_gpu_parity import THREADS, adversarial_sigs, corrupted_single_sets, interop_sks, msg

pytestmark = pytest.mark.gpu


def fresh_ctx():
    from lodestar_amd.native import Context

    return Context([0])


def two_job_call(bad_kind):
    """Two batchable single-set jobs in bytes mode: job 0 carries the defect, job 1 is valid."""
    sks = interop_sks(2, first=7000)
    pks = bytearray(cpu.sk_to_pk(sks, threads=THREADS))
    msgs = [msg(j, b"spec") for j in range(2)]
    sigs = [bytearray(s) for s in (lambda b: [b[:96], b[96:]])(cpu.sign(sks, b"".join(msgs), threads=THREADS))]
    if bad_kind == "not_in_group":
        sigs[0] = bytearray(adversarial_sigs()[bls.BLST_POINT_NOT_IN_GROUP])
    elif bad_kind == "bad_pubkey":
        pks[0] |= 0x80  # compressed flag on a 96-byte key: BLST_BAD_ENCODING for the job
    elif bad_kind == "pubkey_not_on_curve":
        pks[95] ^= 1  # y changed: off the curve
    return dict(job_first_set=[0, 1, 2], sigs=b"".join(bytes(s) for s in sigs), sig_len=[96, 96],
                msgs=b"".join(msgs), pk_bytes=bytes(pks), job_flags=[1, 1], sig_stride=96)


@pytest.mark.parametrize("bad_kind,code", [("not_in_group", bls.BLST_POINT_NOT_IN_GROUP),
                                           ("bad_pubkey", bls.BLST_BAD_ENCODING),
                                           ("pubkey_not_on_curve", bls.BLST_POINT_NOT_ON_CURVE)])
@pytest.mark.parametrize("policy", [0, 1])
def test_speculative_msm_rejected_job_leaves_valid_job_true(bad_kind, code, policy):
    """Idle device (fresh context, first call): the 2-job group's speculative S includes the rejected job's decoded
    signature; the valid job must still verify."""
    call = two_job_call(bad_kind)
    want, _ = cpu.verify_jobs(threads=THREADS, **call)
    assert list(want) == [-code, 1]
    c = fresh_ctx()
    try:
        c.set_option("group_policy", policy)
        got, _ = c.verify_raw(**call)
        assert list(got) == [-code, 1]
        # and a 3-set job whose middle set is the defective one, next to a valid 2-set job
        sks = interop_sks(5, first=7100)
        pks = cpu.sk_to_pk(sks, threads=THREADS)
        msgs = [msg(j, b"spec3") for j in range(5)]
        sg = cpu.sign(sks, b"".join(msgs), threads=THREADS)
        sl = [sg[96 * i: 96 * i + 96] for i in range(5)]
        sl[1] = adversarial_sigs()[bls.BLST_POINT_NOT_IN_GROUP]
        call3 = dict(job_first_set=[0, 3, 5], sigs=b"".join(sl), sig_len=[96] * 5, msgs=b"".join(msgs), pk_bytes=pks,
                     job_flags=[1, 1], sig_stride=96)
        c2 = fresh_ctx()
        try:
            c2.set_option("group_policy", policy)
            got, _ = c2.verify_raw(**call3)
        finally:
            c2.close()
        assert list(got) == [-bls.BLST_POINT_NOT_IN_GROUP, 1]
    finally:
        c.close()


def test_idle_small_run_mixed_defects_vs_oracle():
    """An idle 128-set run (the speculative path) with non-G2 signatures, wrong-message sets and valid sets, in jobs of
    1-3 sets, job for job against the oracle; the same call on a busy device (no speculation) agrees."""
    n = 128
    rng = np.random.default_rng(128)
    sks = interop_sks(n, first=7300)
    pks = cpu.sk_to_pk(sks, threads=THREADS)
    msgs = [msg(j, b"idle") for j in range(n)]
    sg = cpu.sign(sks, b"".join(msgs), threads=THREADS)
    sl = [sg[96 * i: 96 * i + 96] for i in range(n)]
    ng = adversarial_sigs()[bls.BLST_POINT_NOT_IN_GROUP]
    for i in (3, 40, 41, 100):
        sl[i] = ng
    for i in (7, 55, 90):
        msgs[i] = msg(i, b"idle-other")
    sizes = []
    while sum(sizes) < n:
        sizes.append(int(min(n - sum(sizes), rng.integers(1, 4))))
    call = dict(job_first_set=np.concatenate([[0], np.cumsum(sizes)]), sigs=b"".join(sl), sig_len=[96] * n,
                msgs=b"".join(msgs), pk_bytes=pks, job_flags=np.ones(len(sizes)), sig_stride=96)
    want, _ = cpu.verify_jobs(threads=THREADS, **call)
    assert (want == 0).sum() >= 2 and (want == -bls.BLST_POINT_NOT_IN_GROUP).sum() >= 3 and (want == 1).sum() > 30
    for policy in (0, 1):
        c = fresh_ctx()
        try:
            c.set_option("group_policy", policy)
            got, _ = c.verify_raw(**call)
            assert np.array_equal(got, want), (policy, np.nonzero(got != want)[0])
            got2, _ = c.verify_raw(**call)  # the context is idle again: same answer
            assert np.array_equal(got2, want)
        finally:
            c.close()


def test_production_scalars_and_entropy_failure():
    """seed 0 draws the scalars from a fresh OS key per call: results equal the oracle's; with the entropy source
    failing, the call is refused (ERR_ENTROPY, every job rejected) and the next call works."""
    from lodestar_amd import native

    n = 2048
    rng = np.random.default_rng(2048)
    sks, pks, msgs, sigs, sig_len = corrupted_single_sets(n, b"prod", rng)
    batch = dict(job_first_set=np.arange(n + 1), sigs=sigs, sig_len=sig_len, msgs=b"".join(msgs), pk_bytes=pks,
                 job_flags=np.ones(n), sig_stride=192)
    want, _ = cpu.verify_jobs(threads=THREADS, **batch)
    c = fresh_ctx()
    try:
        for _ in range(2):
            got, _ = c.verify_raw(**batch, seed=0)
            assert np.array_equal(got, want)
        native.debug_inject(native.INJECT_ENTROPY, 0, 1)
        try:
            with pytest.raises(RuntimeError, match="ERR_ENTROPY"):
                c.verify_raw(**batch, seed=0)
        finally:
            native.debug_inject(native.INJECT_ENTROPY, 0, 0)
        got, _ = c.verify_raw(**batch, seed=0)
        assert np.array_equal(got, want)
    finally:
        c.close()


def test_device_error_rejects_every_job_and_dispatcher_survives():
    from lodestar_amd import native

    n = 2048
    rng = np.random.default_rng(4096)
    sks, pks, msgs, sigs, sig_len = corrupted_single_sets(n, b"deverr", rng)
    batch = dict(job_first_set=np.arange(n + 1), sigs=sigs, sig_len=sig_len, msgs=b"".join(msgs), pk_bytes=pks,
                 job_flags=np.ones(n), sig_stride=192)
    want, _ = cpu.verify_jobs(threads=THREADS, **batch)
    c = fresh_ctx()
    try:
        # 1. a lone call: every job -DEVICE_ERROR, never 0 or 1
        native.debug_inject(native.INJECT_DEVICE, 0, 1)
        got, _ = c.verify_raw(**batch)
        assert (got == -native.DEVICE_ERROR).all()
        got, _ = c.verify_raw(**batch)
        assert np.array_equal(got, want)
        # 2. calls merged into one failing run: one run in flight at a time, so the calls queued behind the first
        # (a 16k-set call) merge into the second run, which fails; the first run and every later call verify
        c.set_option("pipeline_depth", 1)
        c.set_option("merge_sets", 1 << 20)
        big_n = 16384
        rng2 = np.random.default_rng(16384)
        _, bpks, bmsgs, bsigs, bsl = corrupted_single_sets(big_n, b"deverr-big", rng2)
        big = dict(job_first_set=np.arange(big_n + 1), sigs=bsigs, sig_len=bsl, msgs=b"".join(bmsgs), pk_bytes=bpks,
                   job_flags=np.ones(big_n), sig_stride=192)
        big_want, _ = cpu.verify_jobs(threads=THREADS, **big)
        native.debug_inject(native.INJECT_DEVICE, 1, 1)
        try:
            with ThreadPoolExecutor(8) as pool:
                f_big = pool.submit(c.verify_raw, **big)
                time.sleep(0.003)
                small = [pool.submit(c.verify_raw, **batch) for _ in range(6)]
                got_big, st_big = f_big.result()
                outs = [f.result() for f in small]
        finally:
            native.debug_inject(native.INJECT_DEVICE, 0, 0)
        failed = [(g, s) for g, s in outs if (g == -native.DEVICE_ERROR).any()]
        ok = [(g, s) for g, s in outs if not (g == -native.DEVICE_ERROR).any()]
        if (got_big == -native.DEVICE_ERROR).any():  # the small calls overtook the big one into the first run
            assert (got_big == -native.DEVICE_ERROR).all()
        else:
            assert np.array_equal(got_big, big_want)
        assert failed, "the injected failure hit no call"
        for g, s in failed:
            assert (g == -native.DEVICE_ERROR).all()  # every job of a failed call rejected, none false
        for g, s in ok:
            assert np.array_equal(g, want)
        assert max(s.run_calls for _, s in failed) >= 2 or (got_big == -native.DEVICE_ERROR).all(), \
            "no merged call failed with its run"
        # 3. the dispatcher survived: later calls (alone and concurrent) verify
        with ThreadPoolExecutor(4) as pool:
            for g, _ in pool.map(lambda _: c.verify_raw(**batch), range(4)):
                assert np.array_equal(g, want)
    finally:
        c.close()


def test_slots_change_from_done_callback_is_refused():
    """blsgpu_set_option("slots") from a done callback (a dispatcher thread) would join its own thread;
    it is refused with ERR_ARGS and the runtime keeps working."""
    import ctypes

    from lodestar_amd import native

    lib = native.load()
    c = fresh_ctx()
    try:
        c.set_option("slots", 2)
        n = 64
        sks = interop_sks(n, first=7600)
        pks = cpu.sk_to_pk(sks, threads=THREADS)
        msgs = b"".join(msg(j, b"cb") for j in range(n))
        sigs = cpu.sign(sks, msgs, threads=THREADS)
        b, keep = native.make_batch(np.arange(n + 1), sigs, [96] * n, msgs, pk_bytes=pks, job_flags=np.ones(n))
        res = np.zeros(n, np.int8)
        st = native.Stats()
        seen = {}
        done = threading.Event()

        @native.DONE_CB
        def cb(user, status):
            seen["status"] = status
            seen["rc"] = lib.blsgpu_set_option(c.h, b"slots", 1)
            done.set()

        rc = lib.blsgpu_submit(c.h, ctypes.byref(b), res.ctypes.data, ctypes.byref(st), cb, None)
        assert rc == native.OK
        assert done.wait(60)
        assert seen["status"] == native.OK and seen["rc"] == native.ERR_ARGS
        assert (res == 1).all()
        assert c.get_option("slots") == 2
        got, _ = c.verify_raw(np.arange(n + 1), sigs, [96] * n, msgs, pk_bytes=pks, job_flags=np.ones(n))
        assert (got == 1).all()
    finally:
        c.close()


def test_two_shards_c4_full_size_vs_oracle():
    """Context([0, 0]) (the in-process multi-device path, both shards on device 0) on C4's whole step: 32,768
    aggregate sets over the 2^20-key table, which the concurrent upload fills on both shards; clean and ~1%
    corrupted, job for job against the oracle."""
    from lodestar_amd.native import Context

    c2 = Context([0, 0])
    try:
        assert c2.device_count == 2
        signer = lambda sks, m: cpu.sign(sks, m, threads=THREADS)
        w, n, desc, _ = bench.build_workload(c2, "C4", 0, 1, signer=signer)
        assert n == 32768 and c2.pubkeys_count == 1 << 20  # min over both shards' tables
        table = bench.oracle_table(w)
        call = {k: v for k, v in w.items() if k != "expected" and not k.startswith("_")}
        got, st = c2.verify_raw(**call)
        assert st.devices_used == 2 and (got == 1).all()
        nmsg = len(w["_mkey"])
        m2 = [bench.msg_j(k, 0xC44) for k in w["_mkey"]]
        sg = cpu.sign(b"".join(w["_sk"]), b"".join(m2), threads=THREADS)
        m2, buf, sl, _ = corrupt.corrupt_sets([sg[96 * i: 96 * i + 96] for i in range(nmsg)], m2,
                                              np.random.default_rng(0xC44))
        bad = dict(call, sigs=np.frombuffer(buf, np.uint8), sig_len=np.asarray(sl, np.uint32),
                   msgs=np.frombuffer(b"".join(m2), np.uint8), sig_stride=192)
        got, st = c2.verify_raw(**bad)
        want, _ = cpu.verify_jobs(table=table, threads=THREADS, **bad)
        assert st.devices_used == 2
        assert np.array_equal(got, want), np.nonzero(got != want)[0][:10]
        assert (got != 1).sum() >= 100
    finally:
        c2.close()


def test_eight_shards_c4_full_size_vs_oracle():
    """C4's whole step through EIGHT in-process device contexts on device 0 (Context([0] * 8): eight dispatcher sets,
    eight stream sets, eight table replicas -- the 8-GPU path of one process, on the one device this box has), with
    route_split_sets 4096 so the 32,768-set call splits into 8 shards of 4,096: ~1% corrupted, job for job against the
    oracle."""
    from lodestar_amd.native import Context

    c8 = Context([0] * 8)
    try:
        assert c8.device_count == 8
        c8.set_option("route_split_sets", 4096)
        signer = lambda sks, m: cpu.sign(sks, m, threads=THREADS)
        w, n, desc, _ = bench.build_workload(c8, "C4", 0, 1, signer=signer)
        assert n == 32768 and c8.pubkeys_count == 1 << 20
        table = bench.oracle_table(w)
        call = {k: v for k, v in w.items() if k != "expected" and not k.startswith("_")}
        nmsg = len(w["_mkey"])
        m2 = [bench.msg_j(k, 0xC48) for k in w["_mkey"]]
        sg = cpu.sign(b"".join(w["_sk"]), b"".join(m2), threads=THREADS)
        m2, buf, sl, _ = corrupt.corrupt_sets([sg[96 * i: 96 * i + 96] for i in range(nmsg)], m2,
                                              np.random.default_rng(0xC48))
        bad = dict(call, sigs=np.frombuffer(buf, np.uint8), sig_len=np.asarray(sl, np.uint32),
                   msgs=np.frombuffer(b"".join(m2), np.uint8), sig_stride=192)
        got, st = c8.verify_raw(**bad)
        want, _ = cpu.verify_jobs(table=table, threads=THREADS, **bad)
        assert st.devices_used == 8
        assert np.array_equal(got, want), np.nonzero(got != want)[0][:10]
        assert (got != 1).sum() >= 100 and (got == 1).sum() > 30000
        got, st = c8.verify_raw(**call)
        assert st.devices_used == 8 and (got == 1).all()
    finally:
        c8.close()

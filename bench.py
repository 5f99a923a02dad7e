#!/usr/bin/env python3
"""Benchmark: verified BLS12-381 signature sets / s on MI355X (BASELINE.json metric).

Workload (SURVEY.md 8d, config C2 "gossip attestation flood"): 16,384 single-pubkey signature sets per GPU
per step, each its own batchable job (as gossip attestations reach IBlsVerifier.verifySignatureSets with
{batchable: true}), distinct messages msg_j = SHA-256(LE64(seed) || LE32(j)), interop keys
sk_i = LE(sha256(LE32_32(i))) mod r (reference state-transition/src/util/interop.ts:19-22), pubkeys in the
device-resident table.  Inputs are generated on the GPU before timing (signing kernels) and are resident
in host pinned staging; one step = one blsgpu_verify call = H2D + full verification + per-job results.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C1|C2|C3|C4|C5]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N      (one rank per GPU)

Prints one JSON line (rank 0).  Multi-GPU: each rank verifies its own 16,384 sets (weak scaling, no
collective on the data path; gloo is used only for the barrier and the max-over-ranks of the timing).
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
SEED = 0x4C4F444553544152  # "LODESTAR"
VALU_PEAK_PRODUCTS = 2.9171e13  # measured v_mad_u64_u32 lane-ops/s, profiles/r01_valu_rates.json


def interop_sk(i):
    return int.from_bytes(hashlib.sha256(i.to_bytes(32, "little")).digest(), "little") % R_ORDER


def msg_j(j, seed=SEED):
    return hashlib.sha256(seed.to_bytes(8, "little") + j.to_bytes(4, "little")).digest()


def gen_keys(ctx, n):
    sks = b"".join(interop_sk(i).to_bytes(32, "big") for i in range(n))
    pks, st = ctx.debug_op(8, sks, 32, 96)
    assert (st == 0).all()
    return sks, pks


def gen_sigs(ctx, sk_bytes_list, msgs, signer=None):
    """Signatures sk_i H(msg_i): on the GPU (debug op 7, pinned to the oracle by tests/test_gpu_parity.py), or by
    `signer(sks, msgs)` (the tests pass the C oracle's sign, so the inputs do not come from the device)."""
    if signer is not None:
        return signer(b"".join(sk_bytes_list), b"".join(msgs))
    inp = b"".join(sk + m for sk, m in zip(sk_bytes_list, msgs))
    sigs, st = ctx.debug_op(7, inp, 64, 96)
    assert (st == 0).all()
    return sigs


def message_variant(ctx, w, v):
    """Workload variant v: the same sets, keys and jobs with every message replaced (msg key k -> msg_j(k) under the
    seed SEED + v) and the signatures re-made on the GPU.  Each in-flight step uses its own variant, so no two calls a
    runtime slot merges into one pipeline run share a signing root: the per-run message dedupe cannot skip
    hash_to_G2 or Miller-line work that a stream of distinct calls would have to do."""
    if v == 0:
        return w
    msgs = [msg_j(k, SEED + v) for k in w["_mkey"]]
    sigs = gen_sigs(ctx, w["_sk"], [msg_j(k, SEED + v) for k in w["_skey"]])
    out = dict(w)
    out["msgs"] = np.frombuffer(b"".join(msgs), np.uint8)
    out["sigs"] = np.frombuffer(sigs, np.uint8)
    return out


def build_workload(ctx, config, rank, world=1, n_dev=1, signer=None, sets=0):
    """Returns dict of numpy inputs for verify_raw + description.  n_dev > 1: one call spans n_dev in-process
    devices (the runtime shards it), so C2 carries 16,384 sets per device.  sets > 0 (C1/C2 diagnostics only) overrides
    the call size."""
    if config in ("C1", "C2"):
        n = (sets or (128 if config == "C1" else 16384)) * n_dev
        sks, pks = gen_keys(ctx, n)
        ctx.upload_pubkeys(0, pks)
        mkeys = [rank * n + j for j in range(n)]
        msgs = [msg_j(k) for k in mkeys]
        sk_list = [sks[32 * i : 32 * i + 32] for i in range(n)]
        sigs = gen_sigs(ctx, sk_list, msgs, signer)
        w = dict(_sk=sk_list, _mkey=mkeys, _skey=mkeys,job_first_set=np.arange(n + 1, dtype=np.uint32), sigs=np.frombuffer(sigs, np.uint8),
                 sig_len=np.full(n, 96, np.uint32), msgs=np.frombuffer(b"".join(msgs), np.uint8),
                 set_pk_first=np.arange(n + 1, dtype=np.uint32), pk_index=np.arange(n, dtype=np.uint32),
                 job_flags=np.ones(n, np.uint8), sig_stride=96, _table_pks=pks)
        desc = {"workload": ("C1 reference perf bench shape: 128 random single-pubkey sets per call, 1 set per batchable job"
                             if config == "C1" else
                             "C2 gossip attestation flood: 16384 single-pubkey sets per GPU, 1 set per batchable job"),
                "sets_per_step_per_gpu": n // n_dev, "pubkeys_per_set": 1, "pk_mode": "device table",
                "sig_encoding": "compressed 96 B", "distinct_messages": n}
        return w, n, desc, 1
    if config == "C3":
        n, k = 128, 512
        n_keys = 65536
        sks, pks = gen_keys(ctx, n_keys)
        ctx.upload_pubkeys(0, pks)
        table_pks = pks
        mkeys = [rank * n + j for j in range(n)]
        msgs = [msg_j(k) for k in mkeys]
        agg_sks = []
        for j in range(n):
            s = sum(interop_sk(i) for i in range(512 * j, 512 * j + k)) % R_ORDER
            agg_sks.append(s.to_bytes(32, "big"))
        sigs = gen_sigs(ctx, agg_sks, msgs, signer)
        w = dict(_sk=agg_sks, _mkey=mkeys, _skey=mkeys,job_first_set=np.array([0, n], np.uint32), sigs=np.frombuffer(sigs, np.uint8),
                 sig_len=np.full(n, 96, np.uint32), msgs=np.frombuffer(b"".join(msgs), np.uint8),
                 set_pk_first=np.arange(0, n * k + 1, k, dtype=np.uint32),
                 pk_index=np.arange(n * k, dtype=np.uint32), job_flags=np.zeros(1, np.uint8), sig_stride=96,
                 _table_pks=table_pks)
        desc = {"workload": "C3 block import: 128 aggregate sets x 512 pubkeys (GPU aggregation), one job",
                "sets_per_step_per_gpu": n, "pubkeys_per_set": k, "pk_mode": "device table (65536 keys)"}
        return w, n, desc, k
    if config == "C4":
        return build_c4(ctx, rank, world, signer)
    if config == "C5":
        return build_c5(ctx, rank, signer)
    raise SystemExit(f"unknown config {config}")


def _table_workload(ctx, set_idx, set_mkey, set_sk, job_sizes, job_flags, sign_mkey=None, signer=None):
    """Inputs for a table-mode call: set_idx[i] = pubkey indices of set i, set_sk[i] = its signing key, set i
    claims message msg_j(set_mkey[i]) and is signed over msg_j(sign_mkey[i]) (default: the claimed one)."""
    sign_mkey = set_mkey if sign_mkey is None else sign_mkey
    sk_list = [s.to_bytes(32, "big") for s in set_sk]
    sigs = gen_sigs(ctx, sk_list, [msg_j(k) for k in sign_mkey], signer)
    n = len(set_idx)
    spf = np.concatenate([[0], np.cumsum([len(x) for x in set_idx])]).astype(np.uint32)
    return dict(_sk=sk_list, _mkey=list(set_mkey), _skey=list(sign_mkey), job_first_set=np.concatenate([[0], np.cumsum(job_sizes)]).astype(np.uint32),
                sigs=np.frombuffer(sigs, np.uint8), sig_len=np.full(n, 96, np.uint32),
                msgs=np.frombuffer(b"".join(msg_j(k) for k in set_mkey), np.uint8), set_pk_first=spf,
                pk_index=np.concatenate([np.asarray(x, np.uint32) for x in set_idx]),
                job_flags=np.asarray(job_flags, np.uint8), sig_stride=96)


def build_c4(ctx, rank, world, signer=None):
    """C4 epoch scale: 2^20-validator table (replicated per GPU), 2,048 committees x 16 aggregate
    sets = 32,768 sets, committee = 512 indices with a seed-random 0-10% dropout per set, one message per
    committee, one batchable job per set.  The 32,768 sets are sharded over the ranks by
    lodestar_amd.shard.shard_jobs (strong scaling)."""
    from lodestar_amd.shard import shard_jobs

    n_val, n_comm, per_comm, csize = 1 << 20, 2048, 16, 512
    sk_all = [interop_sk(i) for i in range(4096)]  # keypairsMod-style tiling (reference perf util.ts:49-50)
    sks_b = b"".join(s.to_bytes(32, "big") for s in sk_all)
    pks, st = ctx.debug_op(8, sks_b, 32, 96)
    assert (st == 0).all()
    reps = n_val // 4096
    for r in range(reps):  # validator i has key i mod 4096
        ctx.upload_pubkeys(r * 4096, pks)
    rng = np.random.default_rng(SEED)
    perm = rng.permutation(n_val).astype(np.uint32)
    n_sets = n_comm * per_comm
    jfs_all = np.arange(n_sets + 1, dtype=np.uint32)
    j0, j1 = shard_jobs(jfs_all, world, None)[rank]
    set_idx, set_msg, set_sk = [], [], []
    for s in range(n_sets):
        c = s // per_comm
        members = perm[(c * csize) % n_val : (c * csize) % n_val + csize]
        drop = rng.random(csize) < rng.random() * 0.10
        if not (j0 <= s < j1):
            continue
        idx = members[~drop] if (~drop).any() else members[:1]
        set_idx.append(idx)
        set_msg.append(c)
        set_sk.append(sum(sk_all[int(i) % 4096] for i in idx) % R_ORDER)
    n = len(set_idx)
    w = _table_workload(ctx, set_idx, set_msg, set_sk, [1] * n, [1] * n, signer=signer)
    w["_table_pks"] = pks * reps
    desc = {"workload": f"C4 epoch scale: 32768 aggregate sets (2048 committees x 16, 512-member committees, "
                        f"0-10% dropout) over a 2^20-validator table, sharded {world} way(s)",
            "sets_per_step_per_gpu": n, "total_sets_per_step": n_sets, "pubkeys_per_set": float(np.mean([len(x) for x in set_idx])),
            "pk_mode": "device table (2^20 validators)", "distinct_messages": n_comm, "scaling": "strong"}
    return w, n, desc, int(round(desc["pubkeys_per_set"]))


def build_c5(ctx, rank, signer=None):
    """C5 mixed: 1,024 sets -- 25% proposer (single), 25% deposit-domain (single), 25%
    sync-committee contribution (aggregate <= 128), 25% sync aggregate (aggregate 512) -- in batchable jobs of
    1-3 sets, 1% of sets signed over the wrong message (-> false, invalid-batch fallback path).  Returns the
    expected per-job results in w['expected']."""
    n_keys = 8192
    sks = [interop_sk(i) for i in range(n_keys)]
    pks, st = ctx.debug_op(8, b"".join(s.to_bytes(32, "big") for s in sks), 32, 96)
    assert (st == 0).all()
    ctx.upload_pubkeys(0, pks)
    rng = np.random.default_rng(SEED + rank)
    n = 1024
    set_idx, set_msg, set_sk = [], [], []
    bad = set(rng.choice(n, size=n // 100, replace=False).tolist())
    for s in range(n):
        kind = s % 4
        if kind < 2:
            idx = rng.integers(0, n_keys, 1)
        elif kind == 2:
            idx = rng.choice(n_keys, size=int(rng.integers(1, 129)), replace=False)
        else:
            idx = rng.choice(n_keys, size=512, replace=False)
        set_idx.append(idx.astype(np.uint32))
        set_msg.append(rank * n + s)
        set_sk.append(sum(sks[int(i)] for i in idx) % R_ORDER)
    sign_keys = [rank * n + s + 1_000_000 if s in bad else set_msg[s] for s in range(n)]
    job_sizes = []
    left = n
    while left:
        k = min(left, int(rng.integers(1, 4)))
        job_sizes.append(k)
        left -= k
    w = _table_workload(ctx, set_idx, set_msg, set_sk, job_sizes, [1] * len(job_sizes), sign_mkey=sign_keys,
                        signer=signer)
    w["_table_pks"] = pks
    jfs = w["job_first_set"]
    w["expected"] = np.array([0 if any(s in bad for s in range(jfs[j], jfs[j + 1])) else 1
                              for j in range(len(job_sizes))], np.int8)
    desc = {"workload": "C5 mixed proposer/deposit/sync-contribution/sync-aggregate sets, jobs of 1-3, 1% invalid",
            "sets_per_step_per_gpu": n, "pubkeys_per_set": float(np.mean([len(x) for x in set_idx])),
            "pk_mode": "device table (8192 keys)", "invalid_sets": len(bad), "jobs": len(job_sizes)}
    return w, n, desc, int(round(desc["pubkeys_per_set"]))


def miller_k_of(st):
    """Pairings per Miller accumulator a run used (the runtime picks it by run size when miller_k = 0): the
    op-count key (1, 2, 4, 8) nearest to pairing units / Miller chunks."""
    k = st.pairing_units / max(st.miller_chunks, 1)
    return min((1, 2, 4, 8), key=lambda c: abs(np.log2(c) - np.log2(max(k, 1.0))))


def stage_mults(n_sets, group_count, pubkeys_per_set, miller_k=2, n_messages=None):
    """Algorithmic work per stage in Montgomery multiplications (lodestar_amd/op_counts.json, counted on the
    host build of the same device algorithm by tools/count_ops.py).  The Miller stage is priced as the kernels
    run it: lines once per distinct message, accumulation per chunk of miller_k pairings."""
    with open(os.path.join(ROOT, "lodestar_amd", "op_counts.json")) as fh:
        oc = json.load(fh)
    per_set = {k: v["total"] for k, v in oc["per_set"].items()}
    acc = oc["miller_acc_per_chunk"]
    k = str(miller_k) if str(miller_k) in acc else "2"
    per_set["miller_sets"] = (oc["miller_lines_per_message"] * (n_messages or n_sets) / n_sets
                              + acc[k] / int(k))
    pgs = oc["per_group_per_set"]
    pgf = oc["per_group_fixed"]
    mults = {
        "sig_decode": per_set["sig_decode"] * n_sets,
        "hash_to_g2": per_set["hash_to_g2"] * (n_messages or n_sets),
        "pk_aggregate": oc["pk_aggregate_per_pubkey"] * n_sets * pubkeys_per_set if pubkeys_per_set > 1 else 0.0,
        "pk_finish": per_set["pk_finish"] * n_sets,
        "sig_msm": per_set["sig_msm"] * n_sets + pgf["sig_msm"] * group_count,
        "miller_sets": per_set["miller_sets"] * n_sets,
        "group_reduce": pgs["group_finish"] * n_sets,
        "group_check": (pgf["group_sig_miller"] + pgf["group_finish"]) * group_count,
    }
    return mults, oc["products_per_mul"]


def roofline(runs, n_sets, group_count, pubkeys_per_set, sets_per_s, miller_k=2, n_messages=None, isolated=None):
    """Dominant kernel: algorithmic limb products per launch / its average launch duration, against the measured
    v_mad_u64_u32 peak.  `runs` are the pipeline runs of the TIMED region, each (stage_ms[8], run_sets, groups,
    distinct messages): HIP events on the stream each stage was launched on, recorded by the runtime while the
    bench ran (a slot that merged queued calls times the merged run, so one launch covers run_sets sets).
    Per stage, achieved = sum of its algorithmic products over the runs / sum of its durations.  `pipeline_frac`
    is the whole chip over the timed region: algorithmic products/s at the measured sets/s over the peak."""
    from lodestar_amd.native import STAGES, KERNEL_OF_STAGE

    prod = np.zeros(len(STAGES))
    ms = np.zeros(len(STAGES))
    ppm = 288
    for st_ms, rs, g, nm, mk in runs:
        mults, ppm = stage_mults(rs, g, pubkeys_per_set, mk, nm)
        prod += np.array([mults[k] for k in STAGES]) * ppm
        ms += np.array(st_ms[:len(STAGES)])
    # dominant kernel = the stage with the largest share of the algorithmic work (the stages of a run overlap on
    # three streams and with other slots' runs, so their durations do not add up to the run's)
    best = int(np.argmax(prod))
    achieved = prod[best] / (ms[best] * 1e-3) / 1e12
    n_runs = max(len(runs), 1)
    per_stage = {STAGES[k]: {"ms_per_launch": round(ms[k] / n_runs, 4),
                             "tproducts_per_s": round(prod[k] / max(ms[k] * 1e-3, 1e-12) / 1e12, 3)}
                 for k in range(len(STAGES))}
    # whole chip: the algorithmic products of the timed runs per set they verified (each run priced with the
    # miller_k it used), at the measured sets/s
    run_sets = sum(r[1] for r in runs)
    if run_sets:
        pipe = float(prod.sum()) / run_sets * sets_per_s
        per_set_products = float(prod.sum()) / run_sets
    else:
        mults1, ppm = stage_mults(n_sets, group_count, pubkeys_per_set, miller_k, n_messages)
        per_set_products = sum(mults1.values()) * ppm / n_sets
        pipe = per_set_products * sets_per_s
    out = {
        "bound": "valu-int",
        "kernel": KERNEL_OF_STAGE[best],
        "achieved": round(achieved, 4),
        "peak": round(VALU_PEAK_PRODUCTS / 1e12, 4),
        "unit": "T limb-products/s (32x32->64)",
        "frac": round(achieved * 1e12 / VALU_PEAK_PRODUCTS, 5),
        "traffic": pmc_traffic(KERNEL_OF_STAGE[best], int(round(np.mean([r[1] for r in runs]))) if runs else 0),
        "traffic_source": pmc_source(),
        "launches_timed": len(runs),
        "sets_per_launch": round(float(np.mean([r[1] for r in runs])), 1) if runs else 0,
        "algorithmic_products_per_launch": round(prod[best] / n_runs),
        "avg_launch_ms": round(ms[best] / n_runs, 4),
        "pipeline_products_per_set": round(per_set_products),
        "pipeline_achieved": round(pipe / 1e12, 4),
        "pipeline_frac": round(pipe / VALU_PEAK_PRODUCTS, 5),
        "stages": per_stage,
    }
    if isolated is not None:
        mi, _ = stage_mults(n_sets, group_count, pubkeys_per_set, miller_k, n_messages)
        out["isolated_call"] = {STAGES[k]: {"ms": round(isolated[k], 4),
                                            "tproducts_per_s": round(mi[STAGES[k]] * ppm / max(isolated[k], 1e-9) / 1e9, 3)}
                                for k in range(len(STAGES))}
    return out


PMC_FILE = os.path.join(ROOT, "profiles", "r06_pmc_traffic.json")
# grid work-items per distinct message (C2: one message per set) of the hash stage's launches; k_batch_inv runs one
# lane per INV_K = 16 elements (csrc/k_inv.hip) and twice per stage (before the maps, before the affine conversion),
# k_hash_map two lanes per message (one SSWU map each), k_hash_clear2 a lane pair per message
PMC_ITEMS_PER_UNIT = {"k_hash_map": 2.0, "k_hash_clear2": 2.0, "k_batch_inv": 2.0 / 16}


def pmc_traffic(kernel, n_sets):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes over the driver's own command
    (tools/gpurun/evidence.sh; FETCH_SIZE doubled for the gfx950 half-count of wide reads, WRITE_SIZE as is;
    MI355X_MICROARCH.md HBM section), kept as bytes per grid work-item because the merged runs differ in size, and
    multiplied by the work-items of an n_sets launch; None when no PMC file is committed."""
    if not n_sets or not os.path.exists(PMC_FILE):
        return None
    with open(PMC_FILE) as fh:
        table = json.load(fh)["kernels"]
    # a stage is several launches ("k_a+k_b+..."); k_batch_inv's figure is per launch of either of its two uses
    # (kernels of the stage that the measured command never launched, e.g. the small-run forms, are absent)
    parts = [p for p in kernel.split("+") if p in table and "FETCH_B_per_item" in table[p]]
    if not parts:
        return None
    per_unit = sum((table[p]["FETCH_B_per_item"] + table[p]["WRITE_B_per_item"]) * PMC_ITEMS_PER_UNIT.get(p, 1.0)
                   for p in parts)
    return round(per_unit * n_sets)


def pmc_source():
    """Where `traffic` comes from: the committed PMC file and whether it was measured on the library this process
    loaded (md5 recorded by tools/pmc_to_json.py) -- a stale file is flagged, never silently reused."""
    if not os.path.exists(PMC_FILE):
        return None
    import hashlib

    from lodestar_amd.native import LIB_PATH

    with open(PMC_FILE) as fh:
        want = json.load(fh).get("lib_md5")
    with open(LIB_PATH, "rb") as fh:
        have = hashlib.md5(fh.read()).hexdigest()
    return {"file": os.path.relpath(PMC_FILE, ROOT), "measured_on_this_library": want == have}


BLST_SETS_PER_CORE = 2200.0  # published anchor: ~0.9 ms/set/thread, x2 batched


def thread_cpu():
    """{tid: (thread name, CPU seconds)} of this process's threads (/proc/self/task; the runtime names its dispatcher
    threads blsgpu-slot / blsgpu-urgent and its packing threads blsgpu-pack)."""
    out, tick = {}, os.sysconf("SC_CLK_TCK")
    try:
        for tid in os.listdir("/proc/self/task"):
            try:
                nm = open(f"/proc/self/task/{tid}/comm").read().strip()
                f = open(f"/proc/self/task/{tid}/stat").read().rsplit(")", 1)[1].split()
                out[tid] = (nm, (int(f[11]) + int(f[12])) / tick)
            except (OSError, ValueError, IndexError):
                pass
    except OSError:
        pass
    return out


def host_cpus():
    """The host CPUs this process may use, checked rather than assumed: the affinity mask
    (os.sched_getaffinity), its physical cores (/proc/cpuinfo physical id + core id), and the CPU share the
    launcher grants through OMP_NUM_THREADS (the GPU box exports its per-GPU share there; os.cpu_count() is the
    whole machine).  Threads used = the affinity count, capped by that share when one is set."""
    aff = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count() or 1))
    phys, model, cur = set(), "", {}
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                k, _, v = line.partition(":")
                k, v = k.strip(), v.strip()
                if k == "processor":
                    cur = {"cpu": int(v)}
                elif k in ("physical id", "core id"):
                    cur[k] = v
                    if "physical id" in cur and "core id" in cur and cur["cpu"] in aff:
                        phys.add((cur["physical id"], cur["core id"]))
                elif k == "model name" and not model:
                    model = v
    except OSError:
        pass
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = min(len(aff), share) if share > 0 else len(aff)
    quota = None  # the cgroup's CPU bandwidth limit (cgroup v2 cpu.max "quota period"), in CPUs
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        quota = None if q == "max" else round(int(q) / int(p), 2)
    except (OSError, ValueError):
        pass
    return {"threads": max(1, threads), "affinity_cpus": len(aff), "affinity_physical_cores": len(phys) or None,
            "cpu_share_env": share or None, "cgroup_cpu_quota": quota, "os_cpu_count": os.cpu_count(), "model": model}


def oracle_table(work):
    from oracle import cpu

    return cpu.Table(work["_table_pks"]) if "_table_pks" in work else None


def concat_calls(calls):
    """One batch of several calls' jobs (same pubkey mode): the reference pool keeps all its workers busy with the
    calls in flight, so the all-core baseline verifies enough jobs at once for every thread to hold a request."""
    out = {"sig_stride": calls[0]["sig_stride"]}
    jfs, spf, off, koff = [np.zeros(1, np.uint32)], [np.zeros(1, np.uint32)], 0, 0
    for c in calls:
        jfs.append(np.asarray(c["job_first_set"][1:], np.uint32) + off)
        if c.get("set_pk_first") is not None:
            spf.append(np.asarray(c["set_pk_first"][1:], np.uint32) + koff)
            koff += int(c["set_pk_first"][-1])
        off += int(c["job_first_set"][-1])
    out["job_first_set"] = np.concatenate(jfs)
    if calls[0].get("set_pk_first") is not None:
        out["set_pk_first"] = np.concatenate(spf)
    for k in ("sigs", "sig_len", "msgs", "job_flags", "pk_index", "pk_bytes"):
        if calls[0].get(k) is not None:
            out[k] = np.concatenate([np.asarray(c[k]) for c in calls])
    return out


def cpu_baseline_all_cores(calls, expected, table, hc):
    """The port on every CPU of the affinity mask -- the reference pool's size, os.cpus().length
    (multithread/poolSize.ts:7) -- over as many in-flight calls as give each thread a >= 128-set worker request."""
    from oracle import cpu

    threads = hc["affinity_cpus"]
    n_sets = int(calls[0]["job_first_set"][-1])
    k = max(1, min(len(calls), -(-threads * 128 // max(n_sets, 1)), 65536 // max(n_sets, 1)))
    batch = concat_calls(calls[:k])
    t0 = time.perf_counter()
    res, st = cpu.verify_jobs(table=table, threads=threads, **batch)
    dt = time.perf_counter() - t0
    agree = bool(np.array_equal(res, np.concatenate([expected] * k)))
    return {"value": round(k * n_sets / dt, 2), "unit": "sets/s", "cores": threads, "kind": "port",
            "sample": f"{k} in-flight steps ({k * n_sets} sets, {st.work_requests} worker requests) through "
                      f"oracle/blscpu.c on all {threads} CPUs of the affinity mask "
                      f"({hc['affinity_physical_cores']} physical cores; cgroup CPU quota "
                      f"{hc['cgroup_cpu_quota'] or 'none'}), {dt:.2f} s, results "
                      f"{'identical to' if agree else 'DIFFERENT from'} the GPU's",
            "results_match_gpu": agree,
            "blst_anchor_sets_per_s": BLST_SETS_PER_CORE * (hc["affinity_physical_cores"] or threads)}


def cpu_baseline(call, expected, table, hc):
    """The reference pool restated in C (oracle/blscpu.c: 6 x 64-bit Montgomery, the pool's job split, >= 16-job
    batch chunks and per-job fallback; kind "port") on this host's cores, on the SAME step the GPU times (all of
    its sets, same inputs), with the result checked against the GPU's.  The blst pool itself cannot run here
    (not vendored, no network): its published per-core anchor is reported beside, at the threads used and at the
    physical cores of the affinity mask."""
    from oracle import cpu

    threads = hc["threads"]
    t0 = time.perf_counter()
    res, st = cpu.verify_jobs(table=table, threads=threads, **call)
    dt = time.perf_counter() - t0
    agree = bool(np.array_equal(res, expected))
    n = len(call["sig_len"])
    cores = hc["affinity_physical_cores"] or hc["affinity_cpus"]
    return {"value": round(n / dt, 2), "unit": "sets/s", "cores": threads, "kind": "port",
            "sample": f"the full bench step ({n} sets, {st.work_requests} worker requests of >= 128 sets, "
                      f"batch chunks of >= 16 jobs) through oracle/blscpu.c on {threads} threads of '{hc['model']}', "
                      f"{dt:.2f} s, results {'identical to' if agree else 'DIFFERENT from'} the GPU's",
            "results_match_gpu": agree,
            "host": {k: hc[k] for k in ("affinity_cpus", "affinity_physical_cores", "cpu_share_env", "cgroup_cpu_quota",
                                        "os_cpu_count")},
            "blst_anchor_sets_per_s": BLST_SETS_PER_CORE * threads,
            "blst_anchor_sets_per_s_affinity_cores": BLST_SETS_PER_CORE * cores,
            "blst_anchor": f"{BLST_SETS_PER_CORE:.0f} sets/s/core (reference lodestar.ts:454 ~0.9 ms/set/thread, "
                           f"x2 batched index.ts:44) x {threads} threads used, and x {cores} physical cores of the "
                           f"affinity mask; the blst pool is not runnable offline"}


PARITY_SEED = SEED + 0x5041524954  # "PARIT"
URGENT_SEED = SEED + 0x55524745  # "URGE"


def urgent_calls(ctx, work, n_calls=32):
    """Latency-critical calls (the reference's verifyOnMainThread: the gossip block proposer signature, one set, and
    verifySignatureSet users; chain/validation/block.ts:146, multithread/index.ts:138-151): n_calls calls alternating 1
    and 3 single-pubkey sets, each one job flagged BLSGPU_JOB_URGENT (not batchable), keys from the step's device table,
    fresh signing roots signed on the GPU before timing.  Returns [(sets, call kwargs)]."""
    from lodestar_amd.native import JOB_URGENT

    out = []
    sks, k = work["_sk"], 0
    for c in range(n_calls):
        n = 1 if c % 2 == 0 else 3
        idx = [(k + i) % len(sks) for i in range(n)]
        k += n
        msgs = [msg_j(1_000_000 + c * 4 + i, URGENT_SEED) for i in range(n)]
        sigs = gen_sigs(ctx, [sks[i] for i in idx], msgs)
        out.append((n, dict(job_first_set=np.array([0, n], np.uint32), sigs=np.frombuffer(sigs, np.uint8),
                            sig_len=np.full(n, 96, np.uint32), msgs=np.frombuffer(b"".join(msgs), np.uint8),
                            set_pk_first=np.arange(n + 1, dtype=np.uint32),
                            pk_index=np.array([work["pk_index"][work["set_pk_first"][i]] for i in idx], np.uint32),
                            job_flags=np.array([JOB_URGENT], np.uint8), sig_stride=96)))
    return out


def urgent_probe(ctx, ucalls, stop, every_ms, lat):
    """Submits the urgent calls one after another, every `every_ms`, until `stop` is set; appends (sets, ms, lane)."""
    i = 0
    while not stop.is_set():
        n, kw = ucalls[i % len(ucalls)]
        t1 = time.perf_counter()
        res, st = ctx.verify_raw(**kw, seed=URGENT_SEED)
        lat.append((n, (time.perf_counter() - t1) * 1e3, int(st.urgent_lane)))
        if res[0] != 1:
            raise SystemExit(f"urgent call {i} ({n} sets) verified {res[0]}, expected 1")
        i += 1
        stop.wait(every_ms / 1e3)


def urgent_summary(lat):
    out = {}
    for n in (1, 3):
        x = np.array([ms for k, ms, _ in lat if k == n])
        if len(x):
            out[f"{n}_set"] = {"n": int(len(x)), "p50": round(float(np.percentile(x, 50)), 3),
                               "p99": round(float(np.percentile(x, 99)), 3), "max": round(float(x.max()), 3)}
    out["on_urgent_lane"] = int(sum(u for _, _, u in lat))
    return out


def parity_leg(ctx, work, pool, calls, expected, table, hc, slots):
    """Untimed parity leg of the bench step: the step's sets re-signed by the ORACLE over fresh signing roots, ~1% of
    them corrupted in every way the reference distinguishes (oracle/corrupt.py: wrong message, another set's
    signature, negated, identity, every Signature.fromBytes error class, 48/0-byte, uncompressed), verified on the
    GPU in the middle of 2 x slots + 2 valid in-flight calls (so a slot merges it with them, the timed region's
    shape) and by oracle/blscpu.c on the same batch and seed; per-job mismatches are counted (reference
    multithread.test.ts:89-106, worker.ts:76-98)."""
    from oracle import corrupt, cpu

    t0 = time.perf_counter()
    n = len(work["_mkey"])
    threads = hc["threads"]
    msgs = [msg_j(k, PARITY_SEED) for k in work["_mkey"]]
    sigs = cpu.sign(b"".join(work["_sk"]), b"".join(msgs), threads=threads)
    rng = np.random.default_rng(PARITY_SEED & 0xFFFFFFFF)
    msgs, sig_buf, sig_len, applied = corrupt.corrupt_sets([sigs[96 * i: 96 * i + 96] for i in range(n)], msgs, rng)
    call = {k: v for k, v in work.items() if not k.startswith("_") and k != "expected"}
    call.update(sigs=np.frombuffer(sig_buf, np.uint8), sig_len=np.asarray(sig_len, np.uint32),
                msgs=np.frombuffer(b"".join(msgs), np.uint8), sig_stride=192)
    k = 2 * slots + 2
    valid = [pool.submit(ctx.verify_raw, **calls[1 + i % (len(calls) - 1)], seed=SEED) for i in range(k // 2)]
    fut = pool.submit(ctx.verify_raw, **call, seed=PARITY_SEED)
    valid += [pool.submit(ctx.verify_raw, **calls[1 + (k // 2 + i) % (len(calls) - 1)], seed=SEED) for i in range(k // 2)]
    got, pst = fut.result()
    valid_ok = sum(int(np.array_equal(f.result()[0], expected)) for f in valid)
    want, ost = cpu.verify_jobs(table=table, threads=threads, **call, seed=PARITY_SEED)
    bad = np.nonzero(got != want)[0]
    kinds = {}
    for i, kd in applied.items():
        kinds[kd] = kinds.get(kd, 0) + 1
    return {"jobs": int(len(want)), "mismatches": int(len(bad)), "first_mismatches": [int(x) for x in bad[:8]],
            "classes": corrupt.result_classes(want), "corrupted_sets": len(applied), "corruptions": kinds,
            "run_calls": int(pst.run_calls), "valid_calls_alongside": len(valid), "valid_calls_correct": valid_ok,
            "oracle": f"oracle/blscpu.c verify_jobs ({threads} threads), signatures by oracle/blscpu.c sign",
            "s": round(time.perf_counter() - t0, 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="C2")
    ap.add_argument("--group-sets", type=int, default=1024)
    ap.add_argument("--group-policy", type=int, default=0,
                    help="0 = batch groups of >= group-sets sets; 1 = the reference pool's jobs / requests / chunks")
    ap.add_argument("--inflight", type=int, default=32,
                    help="verifySignatureSets calls in flight per GPU (runtime slots); 1 = strictly serial")
    ap.add_argument("--slots", type=int, default=0,
                    help="runtime slots per GPU (0 = the runtime's default for the process's hardware queues); fewer "
                         "slots than calls in flight make each slot merge the queued calls into one pipeline run")
    ap.add_argument("--merge-sets", type=int, default=131072, help="max sets of one merged pipeline run (0 = never)")
    ap.add_argument("--pipeline-depth", type=int, default=None, help="runs in flight per device (runtime default 2)")
    ap.add_argument("--merge-wait-us", type=int, default=None,
                    help="how long a slot lingers for more calls to merge while runs are in flight (runtime default)")
    ap.add_argument("--idle-wait-us", type=int, default=None,
                    help="on an idle device, how long a slot waits while a burst of calls keeps arriving (runtime default)")
    ap.add_argument("--miller-k", type=int, default=0,
                    help="pairings per Miller accumulator (shared squarings); 0 = the runtime's choice by run size")
    ap.add_argument("--lane-tail-min", type=int, default=-1,
                    help="runs of >= this many sets use lane forms of the signature tails (-1 = runtime default, 0 never)")
    ap.add_argument("--lane-tail-parts", type=int, default=-1, help="bit 0 Horner, bit 1 MillerLoop(-g1, S)")
    ap.add_argument("--merge-balance", type=int, default=-1, help="cut a backlog into equal runs (-1 = default)")
    ap.add_argument("--lines-lanes", type=int, default=0, help="lanes per message of the Miller lines (0 = default)")
    ap.add_argument("--msm-slice-mid", type=int, default=0, help="MSM slice length of 1k-32k-set runs (0 = default)")
    ap.add_argument("--msm-tree", type=int, default=-1, help="pairwise slice tree for those runs (-1 = default)")
    ap.add_argument("--f-run-max", type=int, default=0, help="F tree: longest lane-serial run (0 = runtime default)")
    ap.add_argument("--miller-lanes", type=int, default=0, help="lanes per pairing of one-item Miller chunks (0 = auto)")
    ap.add_argument("--sets", type=int, default=0, help="diagnostics: sets per call of C1/C2 (default the config's)")
    ap.add_argument("--serial", action="store_true",
                    help="diagnostics: every branch of a run on one stream (each kernel alone on the chip)")
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE",
                    help="any other runtime option (blsgpu_set_option), e.g. --set coop_max=1024; repeatable")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--devices-same", type=int, default=-1,
                    help="host-capacity mode: the --gpus N in-process device contexts all on this one device (N "
                         "dispatcher sets and stream sets on one GPU; throughput is one GPU's, the host cost is N's); "
                         "under torch.distributed.run every rank on this device (the multi-process path rehearsed on "
                         "one GPU)")
    ap.add_argument("--urgent-every-ms", type=float, default=0.0,
                    help="latency probe: during the timed region one thread submits urgent 1- / 3-set calls "
                         "(verifyOnMainThread, BLSGPU_JOB_URGENT) this often, and their isolated latency is measured "
                         "before it (0 = off)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist  # control plane only (barrier / max), no data-path collective

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)

    from concurrent.futures import ThreadPoolExecutor

    from lodestar_amd.native import Context

    # one process per GPU under torch.distributed.run; without a launcher, --gpus N uses N devices in-process
    # (each call sharded over them by the runtime)
    n_dev = args.gpus if world == 1 else 1
    devices = list(range(n_dev)) if world == 1 else [local_rank]
    if args.devices_same >= 0:  # rehearsal on fewer GPUs: every in-process device / every rank on this one
        devices = [args.devices_same] * len(devices)
    ctx = Context(devices)
    ctx.set_option("group_sets", args.group_sets)
    ctx.set_option("group_policy", args.group_policy)
    if args.slots:
        ctx.set_option("slots", args.slots)
    ctx.set_option("merge_sets", args.merge_sets)
    ctx.set_option("miller_k", args.miller_k)
    if args.pipeline_depth is not None:
        ctx.set_option("pipeline_depth", args.pipeline_depth)
    if args.merge_wait_us is not None:
        ctx.set_option("merge_wait_us", args.merge_wait_us)
    if args.idle_wait_us is not None:
        ctx.set_option("idle_wait_us", args.idle_wait_us)
    if args.serial:
        ctx.set_option("serial", 1)
    if args.miller_lanes:
        ctx.set_option("miller_lanes", args.miller_lanes)
    if args.f_run_max:
        ctx.set_option("f_run_max", args.f_run_max)
    if args.merge_balance >= 0:
        ctx.set_option("merge_balance", args.merge_balance)
    if args.lines_lanes:
        ctx.set_option("lines_lanes", args.lines_lanes)
    if args.msm_slice_mid:
        ctx.set_option("msm_slice_mid", args.msm_slice_mid)
    if args.msm_tree >= 0:
        ctx.set_option("msm_tree", args.msm_tree)
    if args.lane_tail_parts >= 0:
        ctx.set_option("lane_tail_parts", args.lane_tail_parts)
    if args.lane_tail_min >= 0:
        ctx.set_option("lane_tail_min", args.lane_tail_min)
    for kv in args.set:
        k, _, v = kv.partition("=")
        ctx.set_option(k, int(v))
    work, n_sets, desc, pk_per_set = build_workload(ctx, args.config, rank, world, n_dev, sets=args.sets)
    expected = work.pop("expected", None)
    if expected is None:
        expected = np.ones(len(work["job_first_set"]) - 1, np.int8)
    # one message variant per in-flight call (step i uses variant i mod V, V > calls in flight)
    n_var = max(2, args.inflight + 1)
    t_gen = time.perf_counter()
    variants = [message_variant(ctx, work, v) for v in range(n_var)]
    t_gen = time.perf_counter() - t_gen
    strip = lambda w: {k: v for k, v in w.items() if not k.startswith("_")}
    calls = [strip(w) for w in variants]
    call = calls[0]

    def step(i=0):
        t1 = time.perf_counter()
        res, st = ctx.verify_raw(**calls[i % n_var], seed=SEED)
        lat_ms = (time.perf_counter() - t1) * 1e3
        if not np.array_equal(res, expected):
            bad = np.nonzero(res != expected)[0]
            fields = {k: (list(getattr(st, k)) if k == "stage_ms" else getattr(st, k)) for k, _ in st._fields_}
            # the same call again: the same wrong jobs = wrong inputs (a device-made signature), else a transient
            res2, _ = ctx.verify_raw(**calls[i % n_var], seed=SEED)
            bad2 = np.nonzero(res2 != expected)[0]
            raise SystemExit(f"verification mismatch on {len(bad)} jobs (first {bad[:8]}: got {res[bad[:8]]}, "
                             f"want {expected[bad[:8]]}); call {i}, variant {i % n_var}, run stats {fields}; "
                             f"re-verified: {len(bad2)} mismatches, same jobs {np.array_equal(bad, bad2)}")
        return st, lat_ms

    pool = ThreadPoolExecutor(max_workers=max(1, args.inflight, 4 * ctx.get_option("slots") + 4))
    for _ in range(args.warmup):
        list(pool.map(step, range(max(1, args.inflight))))
    urgent = None
    if args.urgent_every_ms > 0:
        import threading

        ucalls = urgent_calls(ctx, work)
        iso = []
        for i in range(2 * len(ucalls)):  # isolated: nothing else in flight
            n, kw = ucalls[i % len(ucalls)]
            t1 = time.perf_counter()
            res, st = ctx.verify_raw(**kw, seed=URGENT_SEED)
            if i >= 4:  # the first calls build the lane's buffers
                iso.append((n, (time.perf_counter() - t1) * 1e3, int(st.urgent_lane)))
            assert res[0] == 1
        urgent = {"isolated_ms": urgent_summary(iso), "every_ms": args.urgent_every_ms,
                  "urgent_cus": ctx.get_option("urgent_cus"), "urgent_isolate": ctx.get_option("urgent_isolate"),
                  "urgent_lane_option": ctx.get_option("urgent_lane")}
        ulat, ustop = [], threading.Event()
    # the untimed isolated calls below use variant 0

    def barrier():
        if dist is not None:
            dist.barrier()

    try:
        import torch

        sync = torch.cuda.synchronize if torch.cuda.is_available() else (lambda: None)
    except Exception:  # torch is plumbing only; every step is complete when its call returns
        sync = lambda: None
    # per-stage HIP events on each slot's stream, recorded by the runtime during the timed region (roofline)
    if not args.no_profile:
        ctx.set_option("profile", 1)
    # ---- timed region: K steps, up to `inflight` of them on the GPU at once ----
    barrier()
    sync()
    t0 = time.perf_counter()
    cpu0 = time.process_time()  # host CPU seconds of every thread of the process (dispatchers, packing, callers)
    thr0 = thread_cpu()
    w0 = time.monotonic_ns()  # the timed window on CLOCK_MONOTONIC, the clock of rocprofv3's kernel timestamps
    if urgent is not None:
        uthread = threading.Thread(target=urgent_probe, args=(ctx, ucalls, ustop, args.urgent_every_ms, ulat))
        uthread.start()
    results = list(pool.map(step, range(args.steps)))
    if urgent is not None:
        ustop.set()
        uthread.join()
        urgent["under_load_ms"] = urgent_summary(ulat)
    sync()
    barrier()
    dt = time.perf_counter() - t0
    cpu_s = time.process_time() - cpu0
    thr1 = thread_cpu()
    by_thread = {}
    for tid, (nm, c1) in thr1.items():
        by_thread[nm] = by_thread.get(nm, 0.0) + c1 - thr0.get(tid, (nm, 0.0))[1]
    w1 = time.monotonic_ns()
    ctx.set_option("profile", 0)
    stats = [r[0] for r in results]
    # re-checked jobs over the timed calls (a run's count is reported to each of its calls): 0 for an all-valid
    # workload unless a batch group's equation failed for valid sets
    fallback_jobs_timed = int(sum(s.fallback_jobs for s in stats))
    call_lat = np.array([r[1] for r in results])
    from lodestar_amd.shard import max_over_ranks

    dt = max_over_ranks(dt, dist)
    strong = desc.pop("scaling", "weak") == "strong"
    total_sets = (desc["total_sets_per_step"] if strong else n_sets * world) * args.steps
    n_gpus = world * n_dev
    value = total_sets / dt
    # ---- isolated batches (untimed): p50 latency of one call alone, and its per-stage kernel times ----
    lat = []
    for _ in range(3):
        st_iso, l_ms = step()
        lat.append(l_ms)
    groups, n_msgs = st_iso.groups, st_iso.unique_messages  # one call alone: its own groups / distinct messages
    runs_timed = [st for st in stats if st.run_sets > 0]
    out = {
        "metric": "verified signature sets/sec (node)",
        "miller_k": args.miller_k or "auto",
        "value": round(value, 2),
        "unit": "sets/s",
        "n_gpus": n_gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt * 1e3 / args.steps, 3),
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "u32/u64 (28-bit-limb Montgomery integer arithmetic)",
        "data": f"synthetic (interop keys, SHA-256 messages, signatures generated on the GPU before timing; "
                f"{n_var} message variants, one per in-flight call, so merged runs share no signing root)",
        "config": dict(desc, group_sets=args.group_sets, group_policy=args.group_policy,
                       batch_groups_per_step=groups, inflight=args.inflight,
                       slots=ctx.get_option("slots"), hw_queues=ctx.get_option("hw_queues"),
                       merge_sets=args.merge_sets, pipeline_depth=ctx.get_option("pipeline_depth"),
                       merge_wait_us=ctx.get_option("merge_wait_us"), idle_wait_us=ctx.get_option("idle_wait_us"),
                       pipeline_runs_timed=len(runs_timed),
                       parallelism=f"shard-by-job x{n_gpus} ({'one process per GPU' if world > 1 else 'in-process devices'}), no collective"),
        "p50_batch_latency_ms": round(float(np.median(lat)), 3),
        "fallback_jobs_timed": fallback_jobs_timed,
        "spurious_groups": ctx.get_option("spurious_groups"),
        # host cost of the timed region: CPU seconds of the whole process per million sets verified, and each run's
        # host time from its slot taking it to its input copy (blsgpu_stats.host_ms)
        "host": {"cpu_s_per_million_sets": round(cpu_s / (total_sets / 1e6), 4), "process_cpu_s": round(cpu_s, 3),
                 "run_host_ms": {"p50": round(float(np.percentile([st.host_ms for st in runs_timed], 50)), 3),
                                 "p99": round(float(np.percentile([st.host_ms for st in runs_timed], 99)), 3),
                                 "runs": len(runs_timed)} if runs_timed else None,
                 "cpu_s_by_thread": {k: round(v, 3) for k, v in sorted(by_thread.items(), key=lambda kv: -kv[1])[:8]},
                 "devices": devices},
        "call_latency_under_load_ms": {"p50": round(float(np.percentile(call_lat, 50)), 2),
                                       "p99": round(float(np.percentile(call_lat, 99)), 2)},
    }
    if urgent is not None:
        out["urgent"] = urgent
    if not args.no_profile:
        runs = [(list(st.stage_ms[:8]), st.run_sets, st.groups, st.unique_messages // n_dev, miller_k_of(st))
                for st in runs_timed if n_dev == 1]
        ctx.set_option("profile", 1)
        stage_acc = np.zeros(8)
        for _ in range(2):
            st_p = step()[0]
            stage_acc += np.array(st_p.stage_ms[:8])
        ctx.set_option("profile", 0)
        out["roofline"] = roofline(runs, n_sets // n_dev, groups // n_dev, pk_per_set, value / n_gpus,
                                   miller_k_of(st_p), n_msgs // n_dev, isolated=stage_acc / 2)
    if rank == 0 and n_gpus == 1 and not (args.no_cpu_baseline and args.no_parity):
        hc = host_cpus()
        table = oracle_table(work)
        if not args.no_parity:
            out["parity"] = parity_leg(ctx, work, pool, calls, expected, table, hc, ctx.get_option("slots"))
        if not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(call, expected, table, hc)
            if hc["affinity_cpus"] > hc["threads"]:
                out["cpu_baseline"]["all_cores"] = cpu_baseline_all_cores(calls, expected, table, hc)
    out["workload_variants"] = {"count": n_var, "gen_s": round(t_gen, 2)}
    out["timed_window_monotonic_ns"] = [w0, w1]  # tools/occupancy.py --window: the timed steps' kernels in a trace
    if rank == 0:
        print(json.dumps(out), flush=True)
    pool.shutdown()
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

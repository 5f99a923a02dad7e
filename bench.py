#!/usr/bin/env python3
"""Benchmark: verified BLS12-381 signature sets / s on MI355X (BASELINE.json metric).

Workload (SURVEY.md 8d, config C2 "gossip attestation flood"): 16,384 single-pubkey signature sets per GPU
per step, each its own batchable job (as gossip attestations reach IBlsVerifier.verifySignatureSets with
{batchable: true}), distinct messages msg_j = SHA-256(LE64(seed) || LE32(j)), interop keys
sk_i = LE(sha256(LE32_32(i))) mod r (reference state-transition/src/util/interop.ts:19-22), pubkeys in the
device-resident table.  Inputs are generated on the GPU before timing (signing kernels) and are resident
in host pinned staging; one step = one blsgpu_verify call = H2D + full verification + per-job results.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2|C3|C5]
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


def gen_sigs(ctx, sk_bytes_list, msgs):
    inp = b"".join(sk + m for sk, m in zip(sk_bytes_list, msgs))
    sigs, st = ctx.debug_op(7, inp, 64, 96)
    assert (st == 0).all()
    return sigs


def build_workload(ctx, config, rank):
    """Returns dict of numpy inputs for verify_raw + description."""
    if config == "C2":
        n = 16384
        sks, pks = gen_keys(ctx, n)
        ctx.upload_pubkeys(0, pks)
        msgs = [msg_j(rank * n + j) for j in range(n)]
        sigs = gen_sigs(ctx, [sks[32 * i : 32 * i + 32] for i in range(n)], msgs)
        w = dict(job_first_set=np.arange(n + 1, dtype=np.uint32), sigs=np.frombuffer(sigs, np.uint8),
                 sig_len=np.full(n, 96, np.uint32), msgs=np.frombuffer(b"".join(msgs), np.uint8),
                 set_pk_first=np.arange(n + 1, dtype=np.uint32), pk_index=np.arange(n, dtype=np.uint32),
                 job_flags=np.ones(n, np.uint8), sig_stride=96)
        desc = {"workload": "C2 gossip attestation flood: 16384 single-pubkey sets per GPU, 1 set per batchable job",
                "sets_per_step_per_gpu": n, "pubkeys_per_set": 1, "pk_mode": "device table",
                "sig_encoding": "compressed 96 B", "distinct_messages": n}
        return w, n, desc, 1
    if config == "C3":
        n, k = 128, 512
        n_keys = 65536
        sks, pks = gen_keys(ctx, n_keys)
        ctx.upload_pubkeys(0, pks)
        msgs = [msg_j(rank * n + j) for j in range(n)]
        agg_sks = []
        for j in range(n):
            s = sum(interop_sk(i) for i in range(512 * j, 512 * j + k)) % R_ORDER
            agg_sks.append(s.to_bytes(32, "big"))
        sigs = gen_sigs(ctx, agg_sks, msgs)
        w = dict(job_first_set=np.array([0, n], np.uint32), sigs=np.frombuffer(sigs, np.uint8),
                 sig_len=np.full(n, 96, np.uint32), msgs=np.frombuffer(b"".join(msgs), np.uint8),
                 set_pk_first=np.arange(0, n * k + 1, k, dtype=np.uint32),
                 pk_index=np.arange(n * k, dtype=np.uint32), job_flags=np.zeros(1, np.uint8), sig_stride=96)
        desc = {"workload": "C3 block import: 128 aggregate sets x 512 pubkeys (GPU aggregation), one job",
                "sets_per_step_per_gpu": n, "pubkeys_per_set": k, "pk_mode": "device table (65536 keys)"}
        return w, n, desc, k
    raise SystemExit(f"unknown config {config}")


def stage_mults(n_sets, group_count, pubkeys_per_set):
    """Algorithmic work per stage in Montgomery multiplications (lodestar_amd/op_counts.json, counted on the
    host build of the same device algorithm by tools/count_ops.py)."""
    with open(os.path.join(ROOT, "lodestar_amd", "op_counts.json")) as fh:
        oc = json.load(fh)
    per_set = {k: v["total"] for k, v in oc["per_set"].items()}
    pgs = oc["per_group_per_set"]
    pgf = oc["per_group_fixed"]
    mults = {
        "sig_decode": per_set["sig_decode"] * n_sets,
        "hash_to_g2": per_set["hash_to_g2"] * n_sets,
        "pk_aggregate": oc["pk_aggregate_per_pubkey"] * n_sets * pubkeys_per_set if pubkeys_per_set > 1 else 0.0,
        "pk_finish": per_set["pk_finish"] * n_sets,
        "sig_scale": per_set["sig_scale"] * n_sets,
        "miller_sets": per_set["miller_sets"] * n_sets,
        "group_reduce": (pgs["group_sig_miller"] + pgs["group_finish"]) * n_sets,
        "group_check": (pgf["group_sig_miller"] + pgf["group_finish"]) * group_count,
    }
    return mults, oc["products_per_mul"]


def roofline(stage_ms_avg, n_sets, group_count, pubkeys_per_set, sets_per_s):
    """Dominant kernel: algorithmic limb products per launch / its average duration (HIP events on its
    stream, isolated profiled pass) against the measured v_mad_u64_u32 peak.  `pipeline_frac` is the whole
    chip over the timed (pipelined) region: algorithmic products/s at the measured sets/s over the peak."""
    mults, ppm = stage_mults(n_sets, group_count, pubkeys_per_set)
    from lodestar_amd.native import STAGES, KERNEL_OF_STAGE

    best = max(range(len(STAGES)), key=lambda k: stage_ms_avg[k])
    name = STAGES[best]
    ms = stage_ms_avg[best]
    achieved = mults[name] * ppm / (ms * 1e-3) / 1e12
    per_stage = {STAGES[k]: {"ms": round(stage_ms_avg[k], 4),
                             "tproducts_per_s": round(mults[STAGES[k]] * ppm / max(stage_ms_avg[k], 1e-9) / 1e9, 3)}
                 for k in range(len(STAGES))}
    total_products = sum(mults.values()) * ppm
    pipe = total_products / n_sets * sets_per_s
    return {
        "bound": "valu-int",
        "kernel": KERNEL_OF_STAGE[best],
        "achieved": round(achieved, 4),
        "peak": round(VALU_PEAK_PRODUCTS / 1e12, 4),
        "unit": "T limb-products/s (32x32->64)",
        "frac": round(achieved * 1e12 / VALU_PEAK_PRODUCTS, 5),
        "traffic": None,
        "algorithmic_products_per_launch": mults[name] * ppm,
        "pipeline_products_per_step": total_products,
        "pipeline_achieved": round(pipe / 1e12, 4),
        "pipeline_frac": round(pipe / VALU_PEAK_PRODUCTS, 5),
        "stages": per_stage,
    }


def cpu_baseline(work, n_sample=128, chunk=16):
    """Oracle ('port') timed on this host: verifySignatureSetsMaybeBatch over chunks of 16 sets
    (BATCHABLE_MIN_PER_CHUNK, reference worker.ts:17), single thread, pure Python big ints."""
    from oracle import bls12_381 as bls

    sets = []
    for i in range(n_sample):
        pk = bls.sk_to_pk(interop_sk(i))
        sets.append((pk, bytes(work["msgs"][32 * i : 32 * i + 32]), bytes(work["sigs"][96 * i : 96 * i + 96])))
    t0 = time.perf_counter()
    ok = True
    for c in range(0, n_sample, chunk):
        ok &= bls.verify_signature_sets_maybe_batch(sets[c : c + chunk], rng=bls.SplitMix64(SEED + c))
    dt = time.perf_counter() - t0
    assert ok, "oracle rejected the GPU-generated workload"
    return {"value": round(n_sample / dt, 3), "unit": "sets/s", "cores": 1, "kind": "port",
            "sample": f"{n_sample} C2 sets verified as {n_sample // chunk} batches of {chunk} by the pure-Python "
                      f"oracle (oracle/bls12_381.py), {dt:.1f} s; reference blst pool unavailable offline"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="C2")
    ap.add_argument("--group-sets", type=int, default=256)
    ap.add_argument("--inflight", type=int, default=8,
                    help="verifySignatureSets calls in flight per GPU (runtime slots); 1 = strictly serial")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
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

    ctx = Context([local_rank])
    ctx.set_option("group_sets", args.group_sets)
    ctx.set_option("slots", max(1, args.inflight))
    work, n_sets, desc, pk_per_set = build_workload(ctx, args.config, rank)
    call = dict(work)

    def step(_=None):
        res, st = ctx.verify_raw(**call, seed=SEED)
        if not (res == 1).all():
            raise SystemExit(f"verification failed on valid workload: {np.unique(res, return_counts=True)}")
        return st

    pool = ThreadPoolExecutor(max_workers=max(1, args.inflight))  # ctypes releases the GIL inside the call
    for _ in range(args.warmup):
        list(pool.map(step, range(max(1, args.inflight))))

    def barrier():
        if dist is not None:
            dist.barrier()

    try:
        import torch

        sync = torch.cuda.synchronize if torch.cuda.is_available() else (lambda: None)
    except Exception:  # torch is plumbing only; every step is complete when its call returns
        sync = lambda: None
    # ---- timed region: K steps, up to `inflight` of them on the GPU at once ----
    barrier()
    sync()
    t0 = time.perf_counter()
    stats = list(pool.map(step, range(args.steps)))
    sync()
    barrier()
    dt = time.perf_counter() - t0
    groups = stats[-1].groups
    if dist is not None:
        import torch

        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    total_sets = n_sets * args.steps * world
    value = total_sets / dt
    # ---- isolated batches (untimed): p50 latency of one call, and per-stage kernel times ----
    lat = []
    for _ in range(3):
        t1 = time.perf_counter()
        step()
        lat.append((time.perf_counter() - t1) * 1e3)
    out = {
        "metric": "verified signature sets/sec (node)",
        "value": round(value, 2),
        "unit": "sets/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt * 1e3 / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32/u64 (28-bit-limb Montgomery integer arithmetic)",
        "data": "synthetic (interop keys, SHA-256 messages, signatures generated on the GPU before timing)",
        "config": dict(desc, group_sets=args.group_sets, batch_groups_per_step=groups, inflight=args.inflight,
                       parallelism=f"shard-by-set x{world}, no collective"),
        "p50_batch_latency_ms": round(float(np.median(lat)), 3),
    }
    if not args.no_profile:
        ctx.set_option("profile", 1)
        stage_acc = np.zeros(8)
        for _ in range(2):
            stage_acc += np.array(step().stage_ms[:8])
        ctx.set_option("profile", 0)
        out["roofline"] = roofline(stage_acc / 2, n_sets, groups, pk_per_set, value / world)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(work)
    if rank == 0:
        print(json.dumps(out), flush=True)
    pool.shutdown()
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Isolated-call latency and loaded throughput of gossip-shaped calls (C2 shape: one single-pubkey batchable set per
job, distinct messages) across call sizes and runtime-option variants -- the data for the cooperative-form thresholds
(runtime.cpp coop_max / coop_g2_max / coop_excl_max).

    python tools/latency_curve.py --sizes 512,1024,2048 --variants 'base:;coop2k:coop_max=2048,coop_g2_max=2048' \
        [--invalid 0.01] [--inflight 32 --load-steps 200] --out gpurun_out/curve.json

Per (variant, size): p50 / min of `--reps` isolated calls (nothing else in flight) and, with --load-steps, sets/s with
`--inflight` calls in flight (each call its own window of a signed pool; message dedupe off so no merged run skips
work).  --invalid f: that fraction of sets is signed over another message (the fallback path, C5-like), results are
checked against the expected per-job verdicts.  Signatures and keys come from the GPU's own signing ops (debug ops 7/8,
pinned to the oracle by tests/test_gpu_parity.py).
"""
import argparse
import hashlib
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


def msg(j, seed=7):
    return hashlib.sha256(seed.to_bytes(8, "little") + j.to_bytes(4, "little")).digest()


def parse_variants(spec):
    out = []
    for part in filter(None, spec.split(";")):
        name, _, opts = part.partition(":")
        d = {}
        for kv in filter(None, opts.split(",")):
            k, _, v = kv.partition("=")
            d[k] = int(v)
        out.append((name, d))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="256,512,1024,2048,4096,8192,16384")
    ap.add_argument("--variants", default="base:")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--invalid", type=float, default=0.0)
    ap.add_argument("--jobs3", action="store_true", help="jobs of 1-3 sets (C5 job shape) instead of one set each")
    ap.add_argument("--inflight", type=int, default=32)
    ap.add_argument("--load-steps", type=int, default=0)
    ap.add_argument("--pool", type=int, default=32768)
    ap.add_argument("--out", default="")
    args = ap.parse_args()

    from lodestar_amd.native import Context

    sizes = [int(x) for x in args.sizes.split(",")]
    pool_n = max(args.pool, max(sizes))
    ctx = Context([0])
    t0 = time.perf_counter()
    sks = [int.from_bytes(hashlib.sha256(i.to_bytes(32, "little")).digest(), "little") % R_ORDER for i in range(pool_n)]
    skb = [s.to_bytes(32, "big") for s in sks]
    pks, st = ctx.debug_op(8, b"".join(skb), 32, 96)
    assert (st == 0).all()
    ctx.upload_pubkeys(0, pks)
    rng = np.random.default_rng(11)
    bad = rng.random(pool_n) < args.invalid
    msgs = [msg(i) for i in range(pool_n)]
    signed = [msg(i + 10_000_000) if bad[i] else msgs[i] for i in range(pool_n)]
    sigs, st = ctx.debug_op(7, b"".join(k + m for k, m in zip(skb, signed)), 64, 96)
    assert (st == 0).all()
    sigs = np.frombuffer(sigs, np.uint8).reshape(pool_n, 96)
    msga = np.frombuffer(b"".join(msgs), np.uint8).reshape(pool_n, 32)
    gen_s = time.perf_counter() - t0

    def job_sizes(n, r):
        if not args.jobs3:
            return [1] * n
        out, left = [], n
        while left:
            k = min(left, int(r.integers(1, 4)))
            out.append(k)
            left -= k
        return out

    def call_of(n, start):
        idx = (np.arange(n) + start) % pool_n
        js = job_sizes(n, np.random.default_rng(n))
        jfs = np.concatenate([[0], np.cumsum(js)]).astype(np.uint32)
        exp = np.array([0 if bad[idx[jfs[j]:jfs[j + 1]]].any() else 1 for j in range(len(js))], np.int8)
        c = dict(job_first_set=jfs, sigs=sigs[idx].reshape(-1), sig_len=np.full(n, 96, np.uint32),
                 msgs=msga[idx].reshape(-1), set_pk_first=np.arange(n + 1, dtype=np.uint32),
                 pk_index=idx.astype(np.uint32), job_flags=np.ones(len(js), np.uint8), sig_stride=96)
        return c, exp

    results = []
    pool = ThreadPoolExecutor(max_workers=max(args.inflight, 4))
    for name, opts in parse_variants(args.variants):
        saved = {k: ctx.get_option(k) for k in opts}
        for k, v in opts.items():
            ctx.set_option(k, v)
        ctx.set_option("dedupe", 0)
        for n in sizes:
            c, exp = call_of(n, 0)
            res, _ = ctx.verify_raw(**c)
            assert np.array_equal(res, exp), f"{name} n={n}: mismatch on {(res != exp).sum()} jobs"
            lat = []
            for _ in range(args.reps):
                t1 = time.perf_counter()
                res, stt = ctx.verify_raw(**c)
                lat.append((time.perf_counter() - t1) * 1e3)
                assert np.array_equal(res, exp)
            row = {"variant": name, "opts": opts, "sets": n, "p50_ms": round(float(np.median(lat)), 3),
                   "min_ms": round(float(np.min(lat)), 3), "fallback_jobs": int(stt.fallback_jobs),
                   "fallback_miller": int(stt.fallback_miller)}
            if args.load_steps:
                calls = [call_of(n, (v * n) % pool_n) for v in range(args.inflight + 1)]

                def step(i):
                    cc, ee = calls[i % len(calls)]
                    r, _ = ctx.verify_raw(**cc)
                    if not np.array_equal(r, ee):
                        raise SystemExit(f"{name} n={n}: loaded mismatch")

                list(pool.map(step, range(args.inflight)))
                t1 = time.perf_counter()
                list(pool.map(step, range(args.load_steps)))
                dt = time.perf_counter() - t1
                row["load_sets_per_s"] = round(args.load_steps * n / dt, 1)
                row["load_steps"] = args.load_steps
            print(json.dumps(row), flush=True)
            results.append(row)
        ctx.set_option("dedupe", 1)
        for k, v in saved.items():  # back to the runtime defaults for the next variant
            ctx.set_option(k, v)
    out = {"tool": "tools/latency_curve.py", "args": vars(args), "gen_s": round(gen_s, 2), "rows": results}
    if args.out:
        os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
        with open(args.out, "w") as fh:
            json.dump(out, fh, indent=1)
    pool.shutdown()
    ctx.close()


if __name__ == "__main__":
    main()

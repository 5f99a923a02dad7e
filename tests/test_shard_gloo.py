"""Multi-rank host logic on CPU (gloo, world_size 2): the job sharding every rank computes independently
tiles the workload exactly once, is cost-balanced, never splits a job, and the bench's max-over-ranks timing
rule holds.  No data-path collective exists; gloo carries only the checks."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from lodestar_amd.shard import job_costs, max_over_ranks, shard_jobs


def workload(seed=7, n_jobs=997):
    rng = np.random.default_rng(seed)
    sets_per_job = rng.integers(0, 4, n_jobs)  # includes empty jobs
    jfs = np.concatenate([[0], np.cumsum(sets_per_job)])
    pks = rng.integers(1, 513, int(jfs[-1]))  # aggregate sizes up to a committee
    spf = np.concatenate([[0], np.cumsum(pks)])
    return jfs, spf


def test_shard_jobs_single_process_properties():
    jfs, spf = workload()
    for n in (1, 2, 3, 8):
        sh = shard_jobs(jfs, n, spf)
        assert sh[0][0] == 0 and sh[-1][1] == len(jfs) - 1
        assert all(a[1] == b[0] for a, b in zip(sh, sh[1:]))
        cost = job_costs(jfs, spf)
        per = [cost[b] - cost[a] for a, b in sh]
        max_job = max(np.diff(cost))
        assert max(per) - min(per) <= 2 * max_job + 1e-9
    assert shard_jobs([0], 4) == [(0, 0)] * 4  # no jobs


def test_cpp_and_python_shard_rules_agree():
    """The C-ABI blsgpu_shard_jobs (the rule the runtime applies over the devices of one process) and
    lodestar_amd/shard.py (the rule ranks apply under torch.distributed) give identical ranges."""
    from lodestar_amd.native import shard_jobs as cpp_shard

    for seed in range(6):
        jfs, spf = workload(seed, n_jobs=300 + 97 * seed)
        for n in (1, 2, 3, 4, 7, 8):
            assert cpp_shard(jfs, n, spf) == shard_jobs(jfs, n, spf)
            assert cpp_shard(jfs, n) == shard_jobs(jfs, n)
    assert cpp_shard([0], 3) == shard_jobs([0], 3) == [(0, 0)] * 3


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        jfs, spf = workload()
        mine = shard_jobs(jfs, world, spf)[rank]
        from lodestar_amd.native import shard_jobs as cpp_shard

        assert cpp_shard(jfs, world, spf)[rank] == mine
        # every rank gathers every rank's independently computed range
        got = [None] * world
        dist.all_gather_object(got, mine)
        dt = max_over_ranks(0.5 + rank)
        q.put((rank, got, dt))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(120)
def test_shard_gloo_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in range(world)]
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    jfs, spf = workload()
    ranges = res[0][1]
    assert all(r[1] == ranges for r in res)  # all ranks agree
    covered = sorted(j for a, b in ranges for j in range(a, b))
    assert covered == list(range(len(jfs) - 1))  # each job exactly once
    assert all(r[2] == 1.5 for r in res)  # max over ranks


def test_c4_in_process_shard_ranges():
    """bench.py --gpus N --config C4 (in-process): ONE call of the 32,768 aggregate sets of C4 (one batchable job
    per set, committees of 512 with 0-10% dropout), which the runtime splits over the N devices with
    blsgpu_shard_jobs -- strong scaling.  The ranges tile the call, match the rank rule, and give every device
    its 1/N of the sets (the sets cost alike)."""
    from lodestar_amd.native import shard_jobs as cpp_shard

    rng = np.random.default_rng(0x4C4F444553544152)
    n_sets = 2048 * 16
    pks = np.array([512 - int(512 * rng.random() * 0.10 * rng.random()) for _ in range(n_sets)])
    jfs = np.arange(n_sets + 1, dtype=np.uint32)
    spf = np.concatenate([[0], np.cumsum(pks)]).astype(np.uint32)
    for n in (1, 2, 4, 8):
        sh = cpp_shard(jfs, n, spf)
        assert sh == shard_jobs(jfs, n, spf)
        assert sh[0][0] == 0 and sh[-1][1] == n_sets and all(a[1] == b[0] for a, b in zip(sh, sh[1:]))
        sizes = [b - a for a, b in sh]
        assert max(sizes) - min(sizes) <= max(64, n_sets // n // 50), sizes

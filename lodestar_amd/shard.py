"""Host-side sharding of a verifySignatureSets workload over ranks (one process per MI355X).

The path shards by independent units: each job yields its own boolean, so jobs are split
into contiguous ranges balanced by estimated cost (1 per set + 1/256 per aggregated pubkey), never
splitting a job, with no collective on the data path.  This is the same rule the C++ runtime applies to
the devices of one process (lodestar_amd/csrc/runtime.cpp, `cost-balanced contiguous sharding`); the
multi-process bench (bench.py --config C4) and the world_size-2 gloo test use this restatement.
"""
import numpy as np


def job_costs(job_first_set, set_pk_first=None):
    """Prefix sums of per-job cost: cost[j] = cost of jobs [0, j)."""
    jfs = np.asarray(job_first_set, dtype=np.int64)
    per_set = np.ones(int(jfs[-1]), dtype=np.float64)
    if set_pk_first is not None:
        spf = np.asarray(set_pk_first, dtype=np.int64)
        per_set += np.diff(spf) / 256.0
    set_prefix = np.concatenate([[0.0], np.cumsum(per_set)])
    return set_prefix[jfs]


def shard_jobs(job_first_set, n_shards, set_pk_first=None):
    """Contiguous [job_begin, job_end) per shard, cost-balanced; the last shard takes the remainder."""
    cost = job_costs(job_first_set, set_pk_first)
    n_jobs = len(cost) - 1
    out, j0 = [], 0
    for k in range(n_shards):
        if k + 1 == n_shards:
            j1 = n_jobs
        else:
            target = cost[-1] * (k + 1) / n_shards
            # largest j1 >= j0 with cost[j1] <= target
            j1 = max(j0, int(np.searchsorted(cost, target, side="right")) - 1)
        out.append((j0, j1))
        j0 = j1
    return out


def route_call(n_sets, device_load, split_sets=16384, start=0):
    """Which devices a call runs on (the runtime's route_rule, runtime.cpp; C-ABI blsgpu_route_call): k =
    min(devices, max(1, n_sets // split_sets)) -- a call below 2 x split_sets sets runs WHOLE on one device -- chosen
    as the k least loaded, ties broken by distance from `start`, returned in ascending order (shard order)."""
    n = len(device_load)
    if n == 0:
        return []
    k = max(1, min(n, n_sets // max(1, split_sets)))
    order = sorted(range(n), key=lambda d: (device_load[d], (d - start) % n))
    return sorted(order[:k])


def max_over_ranks(dt, dist=None):
    """The bench's timing rule: the slowest rank's wall time (gloo all_reduce MAX; control plane only)."""
    if dist is None:
        import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(dt)
    import torch

    t = torch.tensor([float(dt)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())

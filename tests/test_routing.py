"""The runtime's call routing (C-ABI blsgpu_route_call, pure host code) against its restatement in
lodestar_amd/shard.py route_call: a call below 2 x route_split_sets sets runs whole on the least-loaded device, a
larger one splits over the least-loaded min(devices, sets / route_split_sets) devices (verdict r4: a 16k gossip call
must not become 2k-set shards on 8 GPUs)."""
import numpy as np

from lodestar_amd import native
from lodestar_amd.shard import route_call


def test_cpp_and_python_route_rules_agree():
    rng = np.random.default_rng(5)
    for _ in range(400):
        nd = int(rng.integers(1, 9))
        load = rng.integers(0, 4, nd) * int(rng.choice([1, 256, 4096]))
        n = int(rng.choice([0, 1, 128, 2048, 16383, 16384, 32767, 32768, 65536, 131072, 10 ** 6]))
        split = int(rng.choice([1, 1024, 16384, 32768]))
        start = int(rng.integers(0, 100))
        assert native.route_call(n, load, split, start) == route_call(n, list(load), split, start)


def test_route_properties():
    idle8 = [0] * 8
    assert route_call(16384, idle8) == [0]                      # a gossip call: whole
    assert len(route_call(32768, idle8)) == 2                  # C4's step: split
    assert route_call(131072, idle8) == list(range(8))
    assert route_call(128, [5, 3, 0, 9]) == [2]                # the least loaded device
    assert route_call(40000, [5, 3, 0, 9]) == [1, 2]           # the two least loaded, in shard order
    # equal loads: the rotating start spreads whole calls over the devices
    assert [route_call(100, idle8, start=s)[0] for s in range(8)] == list(range(8))
    assert route_call(10 ** 6, [0, 0]) == [0, 1]               # never more devices than exist
    assert native.route_call(16384, idle8) == [0] and native.route_call(32768, idle8, 16384, 3) == [3, 4]

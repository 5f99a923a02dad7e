"""The reference pool's chunking rule (A5), CPU only: chunkifyMaximizeChunkSize against the reference's own test
table (packages/beacon-node/test/unit/chain/bls/utils.test.ts:7-25, minPerChunk 3 over linspace(0, i)), through the
oracle's restatement (oracle/blscpu.c) and the product's (runtime.cpp, C-ABI blsgpu_chunkify) -- the rule
group_policy 1 applies to calls (128 sets, multithread/index.ts:156) and to a request's batchable jobs (16,
multithread/worker.ts:17,56)."""
import pytest

from lodestar_amd import native
from oracle import cpu

# utils.test.ts:7-25: expected chunks of linspace(0, i) for i = 0..7 with minPerChunk = 3
REFERENCE_TABLE = [
    [[0]],
    [[0, 1]],
    [[0, 1, 2]],
    [[0, 1, 2, 3]],
    [[0, 1, 2, 3, 4]],
    [[0, 1, 2], [3, 4, 5]],
    [[0, 1, 2, 3], [4, 5, 6]],
    [[0, 1, 2, 3], [4, 5, 6, 7]],
]


def reference_rule(length, min_per_chunk):
    """utils.ts:4-19 restated line by line (the table above pins it)."""
    arr = list(range(length))
    count = length // min_per_chunk
    if count <= 1:
        return [arr]
    per = -(-length // count)
    return [arr[i: i + per] for i in range(0, length, per)]


@pytest.mark.parametrize("impl", ["oracle", "product"])
def test_chunkify_reference_table(impl):
    f = cpu.chunkify if impl == "oracle" else native.chunkify
    for i, want in enumerate(REFERENCE_TABLE):
        assert f(i + 1, 3) == want, (impl, i)


@pytest.mark.parametrize("impl", ["oracle", "product"])
def test_chunkify_pool_sizes(impl):
    """The two uses on the path: sets of a call (min 128) and batchable jobs of a request (min 16), including the
    empty array ([arr] = [[]] in the reference)."""
    f = cpu.chunkify if impl == "oracle" else native.chunkify
    for m in (3, 16, 128):
        for n in list(range(0, 300)) + [1000, 4097, 16384]:
            assert f(n, m) == reference_rule(n, m), (impl, n, m)
    # C2 (16,384 sets in one call): 128 jobs of 128 sets
    assert [len(c) for c in f(16384, 128)] == [128] * 128

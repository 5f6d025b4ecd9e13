"""The N>1 path on CPU: world_size-2 gloo process groups drive the same
partition / barrier / max-over-ranks code bench.py uses on RCCL (one process
per GPU).  No GPU: the engine's host-side partitioner is plain C."""
import os
import random
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, lengths, out_dir):
    import torch.distributed as dist

    from speedb_amd import shard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        b, e = shard.rank_range(lengths, len(lengths), world, rank)
        mine = int(sum(lengths[b:e]))
        total = shard.reduce_sum(mine)
        slow = shard.timed_steps(lambda: sum(range(20000 * (rank + 1))), 3)
        mx = shard.reduce_max(float(rank + 1))
        u_b, u_e = shard.rank_range(None, 1000, world, rank, length=4096)
        np.save(os.path.join(out_dir, f"r{rank}.npy"),
                np.array([b, e, mine, total, mx, slow, u_b, u_e], dtype=np.float64))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_partition_and_collectives_gloo(tmp_path, world):
    rnd = random.Random(world)
    lengths = [rnd.choice([4096, 16384, 65536]) + rnd.randrange(0, 256) for _ in range(5000)]
    mp.spawn(_worker, args=(world, _free_port(), lengths, str(tmp_path)), nprocs=world, join=True)
    res = [np.load(tmp_path / f"r{r}.npy") for r in range(world)]
    # contiguous, disjoint, covering
    assert res[0][0] == 0 and res[-1][1] == len(lengths)
    for a, b in zip(res, res[1:]):
        assert a[1] == b[0]
    # byte-balanced within one span of the ideal share
    ideal = sum(lengths) / world
    for r in res:
        assert abs(r[2] - ideal) <= max(lengths)
        assert r[3] == sum(lengths)       # reduce_sum
        assert r[4] == world              # reduce_max
        assert r[5] > 0
    # the max-over-ranks time is the same number on every rank
    assert len({r[5] for r in res}) == 1
    # uniform spans split evenly
    sizes = [r[7] - r[6] for r in res]
    assert sum(sizes) == 1000 and max(sizes) - min(sizes) <= 1


def test_partition_edge_cases():
    from speedb_amd import shard
    assert list(shard.partition_spans([], 0, 4)) == [0, 0, 0, 0, 0]
    assert list(shard.partition_spans([10], 1, 3))[-1] == 1
    f = shard.partition_spans(None, 7, 7, length=1)
    assert list(f) == list(range(8))
    with pytest.raises(Exception):
        shard.partition_spans([1, 2], 3, 2)


def _long_worker(rank, world, port, data, out_dir):
    import ctypes

    import torch.distributed as dist

    from speedb_amd import shard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # this rank's contiguous slice of ONE span; its CRC from the CPU
        # oracle (test infrastructure: no GPU here), rank 0 with an init
        orc = ctypes.CDLL(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                       "oracle", "liboracle.so"))
        orc.orc_crc32c_extend.restype = ctypes.c_uint32
        orc.orc_crc32c_extend.argtypes = [ctypes.c_uint32, ctypes.c_char_p, ctypes.c_size_t]
        cuts = [len(data) * r // world for r in range(world + 1)]
        part = data[cuts[rank]:cuts[rank + 1]]
        init = 0x1234ABCD if rank == 0 else 0
        crc = orc.orc_crc32c_extend(init, part, len(part))
        whole = shard.combine_span_crcs(int(crc), len(part))
        np.save(os.path.join(out_dir, f"l{rank}.npy"), np.array([whole], dtype=np.uint64))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_long_span_split_across_ranks_gloo(tmp_path, world, oracle):
    """one long span split across ranks; the (crc, length)
    pairs are all-gathered (8 B per rank) and folded with Crc32cCombine --
    every rank ends with crc32c::Extend(init, whole span)."""
    rnd = random.Random(40 + world)
    data = bytes(rnd.getrandbits(8) for _ in range(200003))
    mp.spawn(_long_worker, args=(world, _free_port(), data, str(tmp_path)), nprocs=world, join=True)
    want = oracle.Extend(0x1234ABCD, data)
    for r in range(world):
        assert int(np.load(tmp_path / f"l{r}.npy")[0]) == want

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

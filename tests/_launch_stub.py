"""Stub rank for tests/test_bench_launch.py: started by bench.launch_ranks
(torch.distributed.run), it joins a gloo group and does what a bench rank
does around its kernel -- its contiguous share of the batch (shard.rank_range),
the timing barrier, the max-over-ranks time and the sum of the bytes -- then
rank 0 writes what it saw as JSON to argv[1]."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import torch.distributed as dist  # noqa: E402

from speedb_amd import shard  # noqa: E402


def main():
    out, expect = sys.argv[1], int(sys.argv[2])
    dist.init_process_group("gloo")
    world, rank = dist.get_world_size(), dist.get_rank()
    assert world == expect == int(os.environ["WORLD_SIZE"]), (world, expect)
    lengths = [4096 + (i * 37) % 256 for i in range(10_000)]
    lo, hi = shard.rank_range(lengths, len(lengths), world, rank)
    mine = sum(lengths[lo:hi])
    shard.barrier()
    total = shard.reduce_sum(mine)
    tmax = shard.reduce_max(float(rank + 1))
    ranges = [None] * world
    dist.all_gather_object(ranges, (lo, hi))
    if rank == 0:
        with open(out, "w") as f:
            json.dump({"world": world, "ranges": ranges, "total": total, "tmax": tmax,
                       "expect_total": sum(lengths)}, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

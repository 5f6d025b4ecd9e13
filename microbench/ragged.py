#!/usr/bin/env python3
"""Ragged-batch throughput of the general (explicit offsets/lengths) paths:
CRC32C (k_crc) and XXH3 (wave / row drivers) over size distributions, to
separate per-span overheads from load imbalance.

  python microbench/ragged.py [--total-gib 1]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import speedb_amd as S  # noqa: E402

DISTS = {
    "u4096_a16": ([4096], [1.0], 0, 16),
    "u4096_gap5": ([4096], [1.0], 0, 5),
    "u4101": ([4101], [1.0], 0, 0),
    "u16384_gap5": ([16384], [1.0], 0, 5),
    "u65536_gap5": ([65536], [1.0], 0, 5),
    "mixed_nojit_a16": ([4096, 16384, 65536], [.6, .3, .1], 0, 16),
    "mixed_sst": ([4096, 16384, 65536], [.6, .3, .1], 256, 5),
    # same multiset, but span i's size depends only on i // 4096, so the
    # static round-robin over 4096 waves gives every wave identical work
    "mixed_wavebal_a16": ("wavebal", None, 0, 16),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--total-gib", type=float, default=1.0)
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    total = int(args.total_gib * 2**30)
    data = torch.randint(0, 256, (total + (1 << 20),), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev)
    for name, (sizes, p, jit, gap) in DISTS.items():
        rng = np.random.default_rng(1)
        lens, offs, pos = [], [], 0
        pattern = rng.permutation([4096] * 6 + [16384] * 3 + [65536])
        while pos < total:
            if sizes == "wavebal":
                n = int(pattern[(len(lens) // 4096) % len(pattern)])
            else:
                n = int(rng.choice(sizes, p=p) + (rng.integers(0, jit) if jit else 0))
            if gap == 16:
                pos = (pos + 15) & ~15
            offs.append(pos)
            lens.append(n)
            pos += n + (gap if gap != 16 else 0)
        nbytes = sum(lens)
        sp = S.Spans(data, len(lens), offsets=torch.tensor(offs, dtype=torch.int64, device=dev),
                     lengths=torch.tensor(lens, dtype=torch.int32, device=dev))
        o32 = torch.empty(len(lens), dtype=torch.int32, device=dev)
        o64 = torch.empty(len(lens), dtype=torch.int64, device=dev)
        res = []
        for kind, fn in (("crc", lambda: S.crc32c_batch(sp, out=o32, stream=st)),
                         ("xxh3", lambda: S.xxh3_64_batch(sp, out=o64, stream=st))):
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(args.iters):
                fn()
            e1.record(st)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / args.iters
            res.append(f"{kind} {nbytes / (ms * 1e-3) / 1e12:5.2f} TB/s ({ms * 1e3:6.1f} us)")
        print(f"{name:18s} n={len(lens):7d}  " + "  ".join(res), flush=True)


if __name__ == "__main__":
    main()

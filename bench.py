#!/usr/bin/env python3
"""Headline benchmark: CRC32C over 1M x 4 KiB random blocks, device-resident
(BASELINE.json configs[1]); metric "GiB/s checksummed (device-resident)".

One step = one mck_crc32c_batch launch over the rank's whole batch.  With
N > 1 (torchrun, one process per GPU) every rank checksums its own 1M-block
shard -- blocks are independent, so there is no data-path collective
(scaling "weak"); the only collectives are the timing barrier and the
max-over-ranks of the elapsed time.

Printed JSON (rank 0): value = total bytes of all ranks / max-over-ranks wall
time of the K timed steps, in GiB/s; roofline = the CRC kernel's algorithmic
bytes per launch / its average launch time from HIP events on the launch
stream, against the 8 TB/s HBM3E peak; cpu_baseline = the reference's own
crc32c (oracle/_ref, compiled from util/crc32c.cc) on the host cores, rank 0
at N=1 only, on a bounded DRAM-resident sample.
"""
import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "GiB/s checksummed (device-resident), 4–64 KiB blocks; % HBM3E peak"
HBM_PEAK = 8.0e12  # B/s, MI355X_MICROARCH.md


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--blocks", type=int, default=1 << 20)
    p.add_argument("--block-bytes", type=int, default=4096)
    p.add_argument("--kind", choices=["crc32c", "xxh3"], default="crc32c")
    p.add_argument("--cpu-seconds", type=float, default=12.0,
                   help="approximate CPU-baseline budget (0 disables)")
    p.add_argument("--cpu-threads", type=int, default=16)
    p.add_argument("--no-verify", action="store_true")
    return p.parse_args()


def cpu_baseline(args, seconds):
    """The reference's crc32c::Value (util/crc32c.cc crc32c_3way, SSE4.2 +
    PCLMUL) / XXH3_64bits, one block per call, blocks strided across threads,
    over a DRAM-resident 1 GiB sample of distinct random blocks."""
    import numpy as np
    flags = open("/proc/cpuinfo").read()
    name = "libspdb_ref_v4.so" if " avx512f " in flags else "libspdb_ref.so"
    path = os.path.join(REPO, "oracle", "_ref", name)
    kind = "reference"
    if not os.path.exists(path):
        return None
    lib = ctypes.CDLL(path)
    lib.ref_bench.restype = ctypes.c_uint64
    lib.ref_bench.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_size_t,
                              ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                              ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint32)]
    block = args.block_bytes
    nblocks = (1 << 30) // block
    buf = np.random.default_rng(7).integers(0, 256, nblocks * block, dtype=np.uint8)
    threads = args.cpu_threads
    k = 0 if args.kind == "crc32c" else 1
    secs = ctypes.c_double()
    sink = ctypes.c_uint32()
    # calibrate with one pass, then size the run to ~`seconds`
    tot = lib.ref_bench(k, 1, threads, block, 0, buf.ctypes.data, nblocks, 1, ctypes.byref(secs),
                        ctypes.byref(sink))
    passes = max(1, int(seconds / max(secs.value, 1e-6)))
    tot = lib.ref_bench(k, 1, threads, block, 0, buf.ctypes.data, nblocks, passes,
                        ctypes.byref(secs), ctypes.byref(sink))
    model = ""
    for line in flags.splitlines():
        if line.startswith("model name"):
            model = line.split(":", 1)[1].strip()
            break
    return {
        "value": round(tot / secs.value / 2**30, 2), "unit": "GiB/s", "cores": threads,
        "kind": kind,
        "sample": (f"{args.kind} via oracle/_ref/{name} (reference util/crc32c.cc + "
                   f"util/xxhash.cc), {passes} pass(es) over {nblocks} distinct random "
                   f"{block}-B blocks (1 GiB, DRAM-resident), one block per call, blocks "
                   f"strided over {threads} threads, {secs.value:.1f} s; host {model}"),
    }


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    import speedb_amd as S

    count, block = args.blocks, args.block_bytes
    g = torch.Generator(device=dev)
    g.manual_seed(1000 + rank)
    data = torch.randint(0, 256, (count * block + 64,), dtype=torch.uint8, device=dev, generator=g)
    spans = S.Spans.uniform(data, block, count)
    out32 = torch.empty(count, dtype=torch.int32, device=dev)
    out64 = torch.empty(count, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)

    def step():
        if args.kind == "crc32c":
            S.crc32c_batch(spans, out=out32, stream=stream)
        else:
            S.xxh3_64_batch(spans, out=out64, stream=stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / args.steps  # one launch per step
    if world > 1:
        t = torch.tensor([wall], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())

    verified = None
    if not args.no_verify:
        # bit-exact spot check of 64 random blocks against the CPU oracle
        import random

        import numpy as np
        orc = ctypes.CDLL(os.path.join(REPO, "oracle", "liboracle.so"))
        orc.orc_crc32c_value.restype = ctypes.c_uint32
        orc.orc_crc32c_value.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
        orc.orc_xxh3_64.restype = ctypes.c_uint64
        orc.orc_xxh3_64.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
        res = (out32.cpu().numpy().view(np.uint32) if args.kind == "crc32c"
               else out64.cpu().numpy().view(np.uint64))
        verified = True
        for i in random.Random(rank).sample(range(count), 64):
            b = data[i * block:(i + 1) * block].cpu().numpy().tobytes()
            want = orc.orc_crc32c_value(b, block) if args.kind == "crc32c" else orc.orc_xxh3_64(b, block)
            verified &= int(res[i]) == want
        if not verified:
            print("bench: RESULT MISMATCH vs oracle", file=sys.stderr)

    total_bytes = count * block * world * args.steps
    value = total_bytes / wall / 2**30
    out_bytes = 4 if args.kind == "crc32c" else 8
    alg_bytes = count * (block + out_bytes)  # per launch: spans read + results written
    achieved = alg_bytes / (kern_ms * 1e-3)
    roof = {
        "bound": "hbm", "achieved": round(achieved / 1e9, 1), "peak": HBM_PEAK / 1e9,
        "unit": "GB/s", "frac": round(achieved / HBM_PEAK, 4), "traffic": None,
        "kernel": "mck::k_crc<OpCrcValue>" if args.kind == "crc32c" else "mck::k_xxh3<OpX3Value>",
        "kernel_avg_ms": round(kern_ms, 4), "alg_bytes_per_launch": alg_bytes,
    }
    traffic_file = os.path.join(REPO, "profiles", f"traffic_{args.kind}_{block}.json")
    if os.path.exists(traffic_file):
        with open(traffic_file) as f:
            tr = json.load(f)
        if tr.get("blocks") == count:
            roof["traffic"] = tr["hbm_bytes_per_launch"]
            roof["traffic_source"] = os.path.relpath(traffic_file, REPO)

    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        cpu = cpu_baseline(args, args.cpu_seconds)

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "GiB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(wall / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic: torch.randint random bytes generated on-device (device-resident)",
            "config": {
                "workload": (f"{args.kind} over {count} x {block} B random blocks per GPU, "
                             "device-resident (BASELINE.json configs[1])"),
                "blocks_per_gpu": count, "block_bytes": block,
                "parallelism": f"partitioned x{world} (no collective)",
            },
            "roofline": roof, "cpu_baseline": cpu, "verified_vs_oracle": verified,
        }
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Benchmarks of the block-checksum hot path (BASELINE.json).

Default workload (the headline, BASELINE.json configs[1]): CRC32C over
1M x 4 KiB random blocks per GPU, device-resident; metric "GiB/s checksummed
(device-resident)".  Other configs via --workload:

  crc32c   configs[1]  CRC32C, N x B uniform blocks (default 1M x 4 KiB)
  xxh3     configs[1]  same data, XXH3-64
  sst      configs[2]  compaction-shaped 4/16/64 KiB (+0..255 B) SST blocks
                       with 5-byte trailers, format_version 6 context
                       checksums; VerifyBlockChecksum of every block, one
                       kCRC32c image and one kXXH3 image (1 GiB each: ~2 GiB
                       per step) per step
  wal      configs[3]  WAL replay: a fixed global batch of 10M x 32 KiB blocks
                       (one kFullType record each) partitioned over the ranks
                       (strong scaling), ReadPhysicalRecord CRC verify of
                       every record; a rank share larger than the HBM budget
                       (--hbm-budget-gib) is verified as passes over one
                       resident image (305 GiB at N=1 > 288 GB of HBM)
  host     configs[4]  host-resident (pinned) 4300-B SST-sized blocks, the
                       8-GPU share of the 80M-key/1KB-value stream per GPU
                       (2.5M blocks, 10.75 GB), H2D + CRC32C + D2H
                       double-buffered through the GPU; also reports the
                       device-only rate of the same blocks
  file     (8f row 2)  whole-file CRC32C (FileChecksumGenCrc32c) of one 4 GiB
                       device-resident file image: 64 KiB pieces + device
                       Crc32cCombine fold; at N > 1 each rank hashes its
                       contiguous slice and the ranks' (crc, length) pairs
                       are all-gathered and folded (8 bytes per rank)
  walwrite (8f row 3)  device WAL writer: a group commit of 2M records of
                       1000-1100 B (README 1 KB values) fragmented, framed
                       and CRC'd into the log byte stream (mck_wal_write_batch)
  blob     (8f row 3)  blob file verify: 1M records (16 B key, 4 KiB value),
                       header + blob CRC of every record (mck_blob_record_batch)
  kv       (row a12)   per-KV protection of memtable inserts, README shape
                       (16 B key, 1000 B value): ProtectKVO(...).ProtectS(seq)
  walrecover (row a11) WAL recovery's device pass (mck_wal_recover_batch): every
                       physical record's CRC32C and every one-fragment record's
                       XXH3 record_checksum in ONE read of a device-resident
                       4 GiB log (--walrec-shape full32k: configs[3]'s one
                       32761-B kFullType record per block; mix: records of
                       100 B - 4 KiB written by the device writer, whose
                       block-straddling records the step also gathers and
                       hashes); the line also carries the end-to-end
                       mck_wal_recover call (host walk + device + readback)
  walrec   (row a10)   EmitPhysicalRecord's CRC of every WAL record of a 1 GiB
                       group of records of 100-1100 B (README 1 KB values,
                       db/log_writer.cc:263-311), back to back at any byte
                       offset: mck_wal_record_crc_batch
  ragged   (8a a1)     crc32c_batch over ragged spans of --span-min..--span-max
                       bytes (explicit offsets/lengths), 1 GiB per GPU
  blockkv  (8f row 4)  Block::InitializeDataBlockProtectionInfo of 1M
                       uncompressed ~4 KiB data blocks (README 16 B user keys
                       as internal keys, 1000 B values; --kv-value-bytes),
                       protection_bytes_per_key 8: layout + key reassembly
                       + ProtectKV of every entry, one batch per step
  shim     (8b)        latency of one synchronous scalar shim call
                       (mck_crc32c_value_r: H2D + launch + D2H) at 64 B,
                       4 KiB, 32 KiB, 1 MiB vs the reference's crc32c::Value
                       on one host thread
  latency  (8f row 1)  latency of one small VerifyBlockChecksum batch of 1,
                       8, 32, 256 ~4.2 KiB blocks (RetrieveMultipleBlocks),
                       device-resident and pinned, vs the reference on one
                       host thread: the crossover INTEGRATION.md 2.1 cites

One step = one pass of the workload's kernel(s) over the rank's whole batch.
With N > 1 (torchrun, one process per GPU) every rank checksums its own
shard -- blocks are independent, so there is no data-path collective
(scaling "weak"); the only collectives are the timing barrier and the
max-over-ranks of the elapsed time.

Before the W warmup steps the workload runs untimed for --settle-ms (250 ms
by default): the first ~25 back-to-back launches of a streaming kernel run up
to 18 % slow while the GPU's clocks settle, so a short warmup
alone would time the transient.

Printed JSON (rank 0): value = checksummed bytes of all ranks / max-over-ranks
wall time of the K timed steps, in GiB/s; roofline = the dominant kernel's
algorithmic bytes per launch / its average launch time (HIP events on the
launch stream) against the 8 TB/s HBM3E peak; cpu_baseline = the reference's
own crc32c / XXH3 (oracle/_ref, compiled from util/crc32c.cc + util/xxhash.cc)
on the CPUs this process may use (cgroup quota / affinity; "cores"), rank 0
at N=1 only: the
DRAM-resident sample of the GPU's own blocks (value) and db_bench's cache-hot
ChecksumBenchmark loop (tools/db_bench_tool.cc:4392-4412, one 4 KiB 'x'
buffer), with the GPU's per-block results cross-checked on a sample.
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
    p.add_argument("--gpus", type=int, default=None,
                   help="ranks (one process per GPU).  Without WORLD_SIZE in the environment and N > 1, "
                        "bench.py starts N fresh ranks itself (torch.distributed.run, a child process); "
                        "under torchrun it must equal WORLD_SIZE")
    p.add_argument("--host-ndev", type=int, default=0,
                   help="host: devices ONE process drives through mck_host_batch_checksum (0 = the rank's own)")
    p.add_argument("--steps", type=int, default=None, help="timed steps (default 50; host 3)")
    p.add_argument("--warmup", type=int, default=None, help="untimed warmup steps (default 100; host 1)")
    # the first ~25 back-to-back launches (~20 ms) of a streaming kernel run
    # up to 18 % slow while the GPU's power management settles (kernel trace:
    # 0.77 -> 0.90 -> 0.76 ms per launch at 1M x 4 KiB): run the workload
    # untimed for this long before the warmup steps, whatever W is
    p.add_argument("--settle-ms", type=float, default=250.0)
    p.add_argument("--engine-lib", default=None,
                   help="time an alternative build of the engine (A/B runs); the line records its path + sha256")
    p.add_argument("--workload", choices=["crc32c", "xxh3", "sst", "wal", "host", "kv", "file", "walwrite", "blob", "shim", "blockkv",
                            "walrec", "ragged", "latency", "walrecover"], default="crc32c")
    p.add_argument("--walrec-shape", choices=["full32k", "mix"], default="full32k",
                   help="walrecover: one 32761-B record per block (configs[3]) or 100 B - 4 KiB records")
    p.add_argument("--walrec-bytes", type=int, default=4 << 30, help="walrecover: log bytes per GPU")
    p.add_argument("--blocks", type=int, default=1 << 20)
    p.add_argument("--block-bytes", type=int, default=4096)
    p.add_argument("--sst-bytes", type=int, default=1 << 30,
                   help="per SST image (sst); 2 images, ~2 GiB per step as BASELINE.md states.  One image "
                        "is one SST file's VerifyChecksumInBlocks batch: 64/256 MiB points in DESIGN.md 5")
    p.add_argument("--sst-types", choices=["both", "crc32c", "xxh3"], default="both",
                   help="sst: verify both images (configs[2]) or one (per-kernel measurement)")
    p.add_argument("--sst-streams", type=int, choices=[1, 2], default=1,
                   help="sst: verify the two images one after the other on one stream (1) or "
                        "concurrently on two, as two input files of a compaction would be (2)")
    p.add_argument("--wal-blocks", type=int, default=10_000_000,
                   help="32 KiB blocks of the WHOLE job, partitioned over the ranks (wal, configs[3])")
    p.add_argument("--hbm-budget-gib", type=float, default=64.0,
                   help="largest resident WAL image per GPU (wal); a bigger share is verified in passes")
    p.add_argument("--file-bytes", type=int, default=4 << 30, help="file image bytes per GPU (file)")
    p.add_argument("--wal-records", type=int, default=2 << 20, help="logical records per GPU (walwrite)")
    p.add_argument("--wal-len-min", type=int, default=1000, help="smallest record payload (walwrite)")
    p.add_argument("--wal-len-max", type=int, default=1100, help="largest record payload (walwrite)")
    p.add_argument("--blob-records", type=int, default=1 << 20, help="blob records per GPU (blob)")
    p.add_argument("--kvs", type=int, default=1 << 22, help="KVs per GPU (kv)")
    p.add_argument("--kv-value-bytes", type=int, default=1000, help="value bytes (kv, blockkv)")
    p.add_argument("--kv-prot-bytes", type=int, default=8, help="protection_bytes_per_key (blockkv)")
    p.add_argument("--kv-two-pass", action="store_true",
                   help="blockkv: the layout + protect pair (host readback between) instead of the one-pass call")
    p.add_argument("--span-min", type=int, default=100, help="smallest span (walrec, ragged)")
    p.add_argument("--span-max", type=int, default=1100, help="largest span (walrec, ragged)")
    p.add_argument("--span-bytes", type=int, default=1 << 30, help="span bytes per GPU (walrec, ragged)")
    p.add_argument("--span-align", type=int, default=1,
                   help="ragged: span starts rounded up to this multiple (128: no cache line shared by two spans)")
    p.add_argument("--ragged-hash", choices=["crc32c", "xxh3"], default="crc32c",
                   help="ragged: the checksum (xxh3: XXH3_64bits per span, mck_xxh3_64_batch)")
    p.add_argument("--host-blocks", type=int, default=2_500_000,
                   help="pinned 4300-B blocks per GPU (host; configs[4]'s 8-GPU share)")
    p.add_argument("--cpu-seconds", type=float, default=12.0,
                   help="approximate CPU-baseline budget (0 disables)")
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="0 = the CPUs this process may use (cgroup quota / affinity)")
    p.add_argument("--no-verify", action="store_true")
    p.add_argument("--crc-driver", choices=["auto", "rows16", "rows8", "rows4", "rows1", "bh"], default="auto",
                   help="force the ragged CRC driver for every workgroup (A/B measurements; the engine's "
                        "test hook mck_test_set_crc_driver)")
    p.add_argument("--crc-order", choices=["blocked", "interleaved"], default="blocked",
                   help="ragged CRC span order per workgroup (A/B measurements)")
    a = p.parse_args()
    if a.steps is None:
        a.steps = 3 if a.workload == "host" else 50
    if a.warmup is None:
        a.warmup = 1 if a.workload == "host" else 100
    if a.workload == "host":
        a.settle_ms = 0.0
    return a


# whole-round uniform CRC kernel (row-transposed, non-temporal loads)


def _cpu_quota():
    """CPUs the cgroup lets this process use (cpu.max), or None."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def usable_cpus():
    """(CPUs this process may actually use, how that was decided): the
    cgroup CPU quota (cpu.max) when set, capped by the affinity mask; the
    hardware thread count (os.cpu_count()) only when neither limits it."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    q = _cpu_quota()
    if q:
        return max(1, min(aff, int(q))), f"cgroup CPU quota {q}, affinity {aff} CPUs"
    return aff, f"affinity {aff} CPUs (no cgroup quota)"


def cpu_baseline(args, kind, block, sample, gpu_results):
    """The reference's crc32c::Value (util/crc32c.cc crc32c_3way, SSE4.2 +
    PCLMUL) or XXH3_64bits, one block per call (tools/db_bench_tool.cc
    :4392-4412), on os.cpu_count() threads (--cpu-threads):
      value      -- DRAM-resident: a host copy of the first 1 GiB of the GPU's
                    own blocks, blocks strided across threads;
      db_bench   -- the ChecksumBenchmark loop itself: every thread hashes one
                    cache-hot std::string(block, 'x') over and over
                    (BASELINE.json configs[0]).
    Before timing, the reference's per-block results on a sample of blocks
    are compared one by one with the GPU's outputs for the same blocks."""
    import numpy as np
    flags = open("/proc/cpuinfo").read()
    name = "libspdb_ref_v4.so" if " avx512f " in flags else "libspdb_ref.so"
    path = os.path.join(REPO, "oracle", "_ref", name)
    if not os.path.exists(path):
        return None
    lib = ctypes.CDLL(path)
    lib.ref_bench.restype = ctypes.c_uint64
    lib.ref_bench.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_size_t,
                              ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                              ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint32)]
    lib.ref_crc32c_value.restype = ctypes.c_uint32
    lib.ref_crc32c_value.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    lib.ref_xxh3_64.restype = ctypes.c_uint64
    lib.ref_xxh3_64.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    buf = np.ascontiguousarray(sample)
    nblocks = buf.size // block
    # per-block cross-check of the GPU on 4096 blocks spread over the sample
    idx = np.unique(np.linspace(0, nblocks - 1, num=min(4096, nblocks)).astype(np.int64))
    fn = lib.ref_crc32c_value if kind == "crc32c" else lib.ref_xxh3_64
    agree = all(int(fn(buf.ctypes.data + int(i) * block, block)) == int(gpu_results[i]) for i in idx)
    usable, how = usable_cpus()
    threads = args.cpu_threads or usable
    k = 0 if kind == "crc32c" else 1
    secs, sink = ctypes.c_double(), ctypes.c_uint32()
    lib.ref_bench(k, 1, threads, block, 0, buf.ctypes.data, nblocks, 1, ctypes.byref(secs),
                  ctypes.byref(sink))  # calibration pass
    budget = args.cpu_seconds * 0.6
    passes = max(1, int(budget / max(secs.value, 1e-6)))
    tot = lib.ref_bench(k, 1, threads, block, 0, buf.ctypes.data, nblocks, passes,
                        ctypes.byref(secs), ctypes.byref(sink))
    dram = tot / secs.value / 2**30
    dram_secs = secs.value
    # db_bench ChecksumBenchmark: calibrate on 64 MiB per thread, then size
    # bytes_per_thread for the rest of the budget
    per = 64 << 20
    lib.ref_bench(k, 0, threads, block, per, None, 0, 0, ctypes.byref(secs), ctypes.byref(sink))
    per = max(per, int(per * (args.cpu_seconds * 0.4) / max(secs.value, 1e-6)))
    tot0 = lib.ref_bench(k, 0, threads, block, per, None, 0, 0, ctypes.byref(secs), ctypes.byref(sink))
    hot = tot0 / secs.value / 2**30
    model = next((ln.split(":", 1)[1].strip() for ln in flags.splitlines()
                  if ln.startswith("model name")), "")
    return {
        "value": round(dram, 2), "unit": "GiB/s", "cores": threads, "kind": "reference",
        "hw_threads": os.cpu_count(), "cores_basis": how,
        "sample": (f"{kind} via oracle/_ref/{name} (reference util/crc32c.cc + util/xxhash.cc), "
                   f"{passes} pass(es) over the GPU workload's first {nblocks} {block}-B blocks "
                   f"({nblocks * block >> 20} MiB host copy, DRAM-resident), one block per call, "
                   f"blocks strided over {threads} threads = the CPUs this process may use ({how}; "
                   f"the host has {os.cpu_count()} hardware threads), {dram_secs:.1f} s; host {model}"),
        "db_bench_cache_hot": {
            "value": round(hot, 2), "unit": "GiB/s", "threads": threads,
            "sample": (f"tools/db_bench_tool.cc:4392-4412 ChecksumBenchmark loop: one "
                       f"std::string({block}, 'x') per thread, {per >> 20} MiB per thread, "
                       f"{secs.value:.1f} s (BASELINE.json configs[0])"),
        },
        "agrees_with_gpu": agree, "blocks_cross_checked": int(len(idx)),
    }


def _ragged(op, mean_len):
    """The kernel that does a ragged (or, since round 5, uniform) CRC
    batch's work: k_crc_ragged, one launch; its workgroups run the body/head
    driver for spans averaging 4 KiB or more, the row drivers otherwise
    (mean_len: the label once named
    the kernel per driver; the 4th template argument is the small-batch
    instance's flag, false for every batch of more than 64 spans)."""
    return f"mck::k_crc_ragged<{op}, true, true, false>"


def C_wal_verify(im, nblocks, stream):
    """mck_wal_verify_batch over the first nblocks blocks of a WalImage."""
    import speedb_amd as S
    return S.wal_verify_batch(im.data, nblocks * 32768, im.log_number, stream=stream,
                              out=im.results[:nblocks])


class Workload:
    """step() runs one pass; span_bytes = checksummed bytes per step;
    alg_bytes = algorithmic HBM bytes per launch of the dominant kernel;
    check() -> bool verifies results (bit-exact spot checks)."""


def make_workload(args, dev, rank, world):
    import numpy as np
    import torch

    import speedb_amd as S
    from speedb_amd import workloads as W

    stream = torch.cuda.current_stream(dev)
    w = Workload()
    w.launches = 1
    if args.workload in ("crc32c", "xxh3"):
        from speedb_amd import shard
        block = args.block_bytes
        # global batch = blocks x world (weak scaling); this rank's contiguous
        # byte-balanced shard of it
        b, e = shard.rank_range(None, args.blocks * world, world, rank, length=block)
        count = e - b
        data, spans = W.uniform_blocks(count, block, dev, seed=1000 + rank)
        out32 = torch.empty(count, dtype=torch.int32, device=dev)
        out64 = torch.empty(count, dtype=torch.int64, device=dev)
        if args.workload == "crc32c":
            w.step = lambda: S.crc32c_batch(spans, out=out32, stream=stream)
            # every block size on the ragged kernel (round 5 retired the
            # uniform-batch kernel: the body/head and row drivers were faster)
            w.kernel = _ragged("mck::OpCrcValueZ", block)
            w.alg_bytes = count * (block + 4)
        else:
            w.step = lambda: S.xxh3_64_batch(spans, out=out64, stream=stream)
            # uniform batches of >= 3 KiB spans (and >= 16 per CU) run on the
            # wave kernel since round 5 (mck_engine.hip kX3UniformWaveMin),
            # those of <= 512 B since round 6 (lane quads, X3_UNIFORM_QUAD_MAX)
            ncu = torch.cuda.get_device_properties(dev).multi_processor_count
            w.kernel = ("mck::k_xxh3_wave<mck::OpX3Value>" if (block >= 3072 or block <= 512) and count >= 16 * ncu
                        else "mck::k_xxh3<mck::OpX3Value>")
            w.alg_bytes = count * (block + 8)
        w.span_bytes = count * block
        w.desc = (f"{args.workload} over {count} x {block} B random blocks per GPU, device-resident" +
                  (" (BASELINE.json configs[1])" if block == 4096 and args.blocks == 1 << 20 else ""))
        w.cfg = {"blocks_per_gpu": count, "block_bytes": block}

        def check():
            # the bytes and per-block outputs the CPU-baseline leg cross-checks
            n = min(count, (1 << 30) // block)
            res = out32 if args.workload == "crc32c" else out64
            w.results = res[:n].cpu().numpy().view(np.uint32 if args.workload == "crc32c" else np.uint64)
            w.sample = data[:n * block].cpu().numpy()
            return None
        w.check = check
    elif args.workload == "sst":
        types = {"both": (S.ChecksumType.kCRC32c, S.ChecksumType.kXXH3), "crc32c": (S.ChecksumType.kCRC32c,),
                 "xxh3": (S.ChecksumType.kXXH3,)}[args.sst_types]
        imgs = [W.SstImage(args.sst_bytes, t, dev, seed=100 + 2 * rank + (0 if t == S.ChecksumType.kCRC32c else 1))
                for t in types]
        res = {}
        side = torch.cuda.Stream(dev) if args.sst_streams == 2 and len(imgs) == 2 else None
        fork, join = torch.cuda.Event(), torch.cuda.Event()

        def step():
            if side is None:
                for im in imgs:
                    res[im.checksum_type] = im.verify(stream=stream)
                return
            # two files at once: the second on a side stream (its workgroups
            # take the CUs the first kernel's tail leaves idle), joined back
            fork.record(stream)
            side.wait_event(fork)
            res[imgs[0].checksum_type] = imgs[0].verify(stream=stream)
            res[imgs[1].checksum_type] = imgs[1].verify(stream=side)
            join.record(side)
            stream.wait_event(join)
        w.step = step
        w.launches = len(imgs)
        w.kernel = " + ".join({int(S.ChecksumType.kCRC32c): _ragged("mck::OpCrcBlock<2>", 1 << 20),
                               int(S.ChecksumType.kXXH3): "mck::k_xxh3_wave<mck::OpX3Block<2> >"}[int(t)]
                              for t in types)
        w.span_bytes = sum(im.payload_bytes + im.count for im in imgs)  # payload + type byte
        # per launch, SURVEY.md 8(d): span bytes (payload + type byte) + the
        # 4 B stored checksum read + the outputs written (1 B mismatch flag,
        # 4 B computed, 4 B stored); descriptors are not counted
        w.alg_bytes = sum(im.payload_bytes + im.count * (1 + 4 + 1 + 4 + 4)
                          for im in imgs) / len(imgs)
        w.desc = ("VerifyBlockChecksum over a compaction-shaped run of 4/16/64 KiB (+0..255 B) SST "
                  f"blocks, {args.sst_bytes >> 20} MiB per image, format_version 6 context "
                  "checksums; " + ("one kCRC32c + one kXXH3 image per step" if len(imgs) == 2 else "one image per step") +
                  (" (BASELINE.json configs[2])" if len(imgs) == 2 and args.sst_bytes == 1 << 30 else ""))
        w.cfg = {"blocks_per_gpu": sum(im.count for im in imgs), "image_bytes": args.sst_bytes,
                 "checksum_types": [S.ChecksumType(int(t)).name for t in types]}
        if side is not None:
            w.cfg["streams"] = 2

        def check():
            # every block the write-side kernel sealed verifies, and injected
            # corruption is flagged exactly
            import random
            ok = True
            for im in imgs:
                mm, _, _, cnt = im.verify(stream=stream, with_count=True)
                ok &= int(cnt.item()) == 0 and int(mm.sum().item()) == 0
                bad = sorted(random.Random(rank).sample(range(im.count), max(1, im.count // 1000)))
                im.corrupt(bad)
                mm, _, _, cnt = im.verify(stream=stream, with_count=True)
                flagged = torch.nonzero(mm).flatten().cpu().tolist()
                im.corrupt(bad)  # restore
                ok &= flagged == bad and int(cnt.item()) == len(bad)
            return ok
        w.check = check
    elif args.workload == "wal":
        from speedb_amd import shard
        # configs[3]: a FIXED global batch partitioned over the ranks (strong
        # scaling, db/db_impl/db_impl_open.cc:1204-1221 replays the logs
        # record by record); a share larger than the HBM budget is verified
        # as passes over one resident image of `res` blocks -- every pass
        # re-reads the image from HBM (64 GiB >> the 256 MB of MALL/L2)
        b, e = shard.rank_range(None, args.wal_blocks, world, rank, length=32768)
        share = e - b
        res = max(1, min(share, int(args.hbm_budget_gib * 2**30) // 32768))
        im = W.WalImage(res, dev, seed=300 + rank)
        passes = [res] * (share // res) + ([share % res] if share % res else [])
        out = {}

        def step():
            for nb in passes:
                out["r"] = C_wal_verify(im, nb, stream)
        w.step = step
        w.launches = len(passes)
        w.scaling = "strong"
        w.kernel = "mck::k_wal_verify<true>"
        w.span_bytes = share * (W.WalImage.PAYLOAD + 1)  # CRC span: type + payload
        # per launch (a full pass): the image + 16 B of result per block
        w.alg_bytes = res * (32768 + 16)
        w.kern_scale = sum(passes) / (res * len(passes))  # partial last pass
        w.desc = (f"WAL replay: {args.wal_blocks} x 32 KiB blocks in the whole job, this rank's share "
                  f"{share} ({share * 32768 / 2**30:.0f} GiB) verified as {len(passes)} pass(es) over a "
                  f"resident {res}-block image, one kFullType 32761-B record per block, "
                  "ReadPhysicalRecord CRC32C verify (BASELINE.json configs[3])")
        w.cfg = {"blocks_total": args.wal_blocks, "blocks_per_gpu": share, "resident_blocks": res,
                 "passes": len(passes), "block_bytes": 32768}

        def check():
            r = C_wal_verify(im, res, stream).cpu()
            return bool((r[:, 0] == 1).all() and (r[:, 1] == 0).all())
        w.check = check
    elif args.workload == "walrecover":
        from speedb_amd import _lib
        log_number = 7
        if args.walrec_shape == "full32k":
            nblocks = args.walrec_bytes // 32768
            im = W.WalImage(nblocks, dev, seed=900 + rank, log_number=log_number)
            img_dev, nbytes = im.data, im.nbytes
            nrec = nblocks
        else:
            rng = np.random.default_rng(900 + rank)
            n = int(args.walrec_bytes // 2100)
            lens = rng.integers(100, 4097, size=n).astype(np.int64)
            offs = np.zeros(n, np.int64)
            offs[1:] = np.cumsum(lens)[:-1]
            src = W.rand_bytes(int(lens.sum()) + 64, dev, 901 + rank)
            log = S.WalBatchWriter(log_number).AddRecords(src, offs, lens)
            nbytes = int(log.numel())
            img_dev = torch.zeros(nbytes + 64, dtype=torch.uint8, device=dev)
            img_dev[:nbytes] = log
            del log, src
            nrec = n
        host_img = img_dev[:nbytes].cpu().numpy().tobytes()
        # the host plan (untimed setup, as mck_wal_recover builds it): every
        # physical record, and the reader's walk for the fragmented records
        t_plan = time.perf_counter()
        plan = S.wal_plan_records(host_img, log_number)
        rplan = S.wal_read_records(host_img, log_number, 0, None)
        walk_s = time.perf_counter() - t_plan
        nphys = len(plan)
        d_plan = torch.from_numpy(plan.view(np.int32)).to(dev)
        ok = torch.empty(nphys, dtype=torch.uint8, device=dev)
        hashes = torch.empty(nphys, dtype=torch.int64, device=dev)
        # fragmented records: their fragments, gathered and hashed in the step
        fr = rplan.frags
        dst = np.array([f.dst_off for f in fr[:rplan.nfrags]], dtype=np.int64)
        typ = np.array([f.type for f in fr[:rplan.nfrags]], dtype=np.int64)
        first = np.searchsorted(dst, rplan.rec_offsets.astype(np.int64))
        nxt = np.append(first[1:], rplan.nfrags)
        multi = [r for r in range(len(first)) if nxt[r] - first[r] > 1 or typ[first[r]] not in (1, 5)]
        mfr, moffs, mlens, mb = [], [], [], 0
        for r in multi:
            moffs.append(mb)
            mlens.append(int(rplan.rec_lengths[r]))
            for j in range(first[r], nxt[r]):
                f = fr[j]
                mfr.append(S.mck_wal_fragment(f.src_off, mb + (f.dst_off - int(rplan.rec_offsets[r])), f.length,
                                              f.type, 0, 0))
            mb += (int(rplan.rec_lengths[r]) + 15) & ~15
        nm = len(multi)
        if nm:
            arr = (S.mck_wal_fragment * len(mfr))(*mfr)
            d_mfr = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(dev)
            gbuf = torch.empty(mb + 64, dtype=torch.uint8, device=dev)
            msp = S.Spans(gbuf, nm, offsets=torch.tensor(moffs, dtype=torch.int64, device=dev),
                          lengths=torch.tensor(mlens, dtype=torch.int32, device=dev))
            mh = torch.empty(nm, dtype=torch.int64, device=dev)

        def step():
            S.wal_recover_batch(img_dev, d_plan, log_number, ok=ok, hashes=hashes, stream=stream)
            if nm:
                _lib.check(_lib.lib.mck_wal_gather_batch(img_dev.data_ptr(), d_mfr.data_ptr(), len(mfr),
                                                         gbuf.data_ptr(), stream.cuda_stream), "mck_wal_gather_batch")
                S.xxh3_64_batch(msp, out=mh, stream=stream)
        w.step = step
        w.launches = 1
        w.span_bytes = nbytes
        # what recovery must move: the log once, the 16-B plan entry, the
        # 1-B verdict and the 8-B record_checksum of every physical record
        w.alg_bytes = nbytes + nphys * (16 + 1 + 8)
        w.kernel = ("mck::k_wal_recover<true>" if not nm else
                    "mck::k_wal_recover<true> + k_wal_gather + mck::k_xxh3 (whole step)")
        shape = ("one kFullType 32761-B record per 32 KiB block (BASELINE.json configs[3] layout)"
                 if args.walrec_shape == "full32k" else
                 f"{nrec} records of 100-4096 B (device writer), {nm} of them block-straddling (gathered + hashed)")
        w.desc = (f"WAL recovery device pass: {nbytes / 2**30:.2f} GiB log per GPU, {shape}; CRC32C of every "
                  "physical record + XXH3 record_checksum from the same registers (mck_wal_recover_batch)")
        w.cfg = {"shape": args.walrec_shape, "log_bytes": nbytes, "records": int(nrec), "physical_records": nphys,
                 "multi_fragment": nm}

        def check():
            okv = bool((ok == 1).all().item())
            hv = hashes.cpu().numpy().view(np.uint64)
            rng = np.random.default_rng(rank)
            # sampled one-fragment records against the engine's scalar
            # XXH3_64bits (another kernel) over the same bytes
            full = np.nonzero((plan[:, 1] >> 24) & 1)[0]
            for k in rng.choice(full, size=min(64, len(full)), replace=False):
                po = int(plan[k, 0]) | ((int(plan[k, 1]) & 0xFFFF) << 32)
                okv &= int(hv[k]) == S.XXH3_64bits(host_img[po:po + int(plan[k, 2])])
            # end-to-end: mck_wal_recover (host walks + device pass + readback)
            reps = 3
            t0 = time.perf_counter()
            infos = []
            for _ in range(reps):
                r = S.WalRecover(host_img, log_number, 0, wal_dev=img_dev)
                infos.append(r.info)
            e2e = (time.perf_counter() - t0) / reps
            okv &= len(r.record_checksums) == nrec and r.dropped_bytes == 0
            w.end_to_end = {
                "value": round(nbytes / e2e / 2**30, 2), "unit": "GiB/s", "seconds": round(e2e, 4),
                "host_walk_s": round(sum(i.walk_seconds for i in infos) / reps, 4),
                "device_s": round(sum(i.device_seconds for i in infos) / reps, 4),
                "records_in_place": int(infos[0].in_place), "records_gathered": int(infos[0].gathered),
                "plan_setup_s": round(walk_s, 4),
                "note": "mck_wal_recover on the device-resident log + its host copy: the host block walk and "
                        "ReadRecord walk (one thread), the plan upload, the device pass, the readback of "
                        "verdicts and checksums; the python wrapper's result copies included"}
            return okv
        w.check = check
    elif args.workload == "file":
        from speedb_amd import shard
        nbytes = args.file_bytes + 4093  # an odd tail: one partial piece
        data = W.rand_bytes(nbytes + 64, dev, 500 + rank)
        scratch = torch.empty(int(S._lib.lib.mck_crc32c_long_scratch_words(nbytes)), dtype=torch.int32,
                              device=dev)
        out = torch.empty(1, dtype=torch.int32, device=dev)
        res = {}

        def step():
            S.crc32c_long(data, nbytes, 0, scratch=scratch, out=out, stream=stream)
            if world > 1:  # the one real exchange: (crc, length) per rank
                res["crc"] = shard.combine_span_crcs(out, nbytes, dev)
        w.step = step
        # 64 KiB pieces on k_crc_ragged (body/head), then k_crc_combine
        w.kernel = _ragged("mck::OpCrcValueZ", 65536)
        w.span_bytes = nbytes
        w.alg_bytes = (nbytes // 65536) * (65536 + 4)
        w.desc = (f"whole-file CRC32C (FileChecksumGenCrc32c, util/file_checksum_helper.h) of a "
                  f"{nbytes}-byte device-resident file image per GPU: 64 KiB pieces + device "
                  "Crc32cCombine fold (SURVEY.md 8f row 2)")
        w.cfg = {"file_bytes_per_gpu": nbytes, "piece_bytes": 65536}

        def check():
            # the long-span result == the host Crc32cCombine fold of the piece
            # CRCs the batch kernel wrote into scratch (two paths agree)
            pieces = scratch.cpu().numpy().view(np.uint32).tolist()
            acc, left = 0, nbytes
            for v in pieces:
                ln = min(65536, left)
                acc = S.crc32c.Crc32cCombine(acc, v, ln)
                left -= ln
            return acc == int(out.cpu().numpy().view(np.uint32)[0])
        w.check = check
    elif args.workload in ("walrec", "ragged"):
        rng = np.random.default_rng(800 + rank)
        n_est = int(args.span_bytes // ((args.span_min + args.span_max) / 2))
        lens = rng.integers(args.span_min, args.span_max + 1, size=n_est).astype(np.int64)
        gaps = rng.integers(0, 8, size=n_est) if args.workload == "walrec" else np.zeros(n_est, np.int64)
        # walrec: a WAL payload follows its 7-byte header (+ trailer gaps):
        # records at any byte offset; ragged: spans back to back
        step = lens + (7 + gaps if args.workload == "walrec" else 0)
        if args.workload == "ragged" and args.span_align > 1:  # each span's slot rounded up
            step = (step + args.span_align - 1) // args.span_align * args.span_align
        offs = np.zeros(n_est, dtype=np.int64)
        offs[1:] = np.cumsum(step)[:-1]
        count = n_est
        data = W.rand_bytes(int(offs[-1] + lens[-1]) + 64, dev, 801 + rank)
        sp = S.Spans(data, count, offsets=torch.from_numpy(offs).to(dev),
                     lengths=torch.from_numpy(lens.astype(np.int32)).to(dev))
        x3 = args.workload == "ragged" and args.ragged_hash == "xxh3"
        out = torch.empty(count, dtype=torch.int64 if x3 else torch.int32, device=dev)
        if args.workload == "walrec":
            types = torch.from_numpy(rng.choice([1, 2, 3, 4], size=count).astype(np.uint8)).to(dev)
            w.step = lambda: S.wal_record_crc_batch(sp, types, 7, out=out, stream=stream)
            w.kernel = _ragged("mck::OpCrcWal", float(lens.mean()))
            w.desc = (f"WAL record CRCs (EmitPhysicalRecord, db/log_writer.cc:263-311): {count} records of "
                      f"{args.span_min}-{args.span_max} B per GPU at any byte offset, mck_wal_record_crc_batch")
        elif x3:
            w.step = lambda: S.xxh3_64_batch(sp, out=out, stream=stream)
            w.kernel = "mck::k_xxh3_wave<mck::OpX3Value>"
            w.desc = (f"xxh3_64_batch over {count} ragged spans of {args.span_min}-{args.span_max} B per GPU "
                      "(explicit offsets/lengths)")
        else:
            w.step = lambda: S.crc32c_batch(sp, out=out, stream=stream)
            w.kernel = _ragged("mck::OpCrcValueZ", float(lens.mean()))
            w.desc = (f"crc32c_batch over {count} ragged spans of {args.span_min}-{args.span_max} B per GPU "
                      "(explicit offsets/lengths)")
        w.span_bytes = int(lens.sum())
        # span bytes + 8 B offset + 4 B length + 4 B out (8 B for XXH3) (+1 B type)
        w.alg_bytes = int(lens.sum()) + count * (16 + (1 if args.workload == "walrec" else 0) + (4 if x3 else 0))
        w.cfg = {"spans_per_gpu": count, "span_min": args.span_min, "span_max": args.span_max}
        if x3:
            w.cfg["hash"] = "xxh3"
        if args.workload == "ragged" and args.span_align > 1:
            w.cfg["span_align"] = args.span_align

        def check():
            idx = np.random.default_rng(rank).choice(count, size=256, replace=False)
            hd = data.cpu().numpy()
            res = out.cpu().numpy().view(np.uint64 if x3 else np.uint32)
            tys = types.cpu().numpy() if args.workload == "walrec" else None
            ok = True
            for k in idx:
                b = hd[offs[k]:offs[k] + lens[k]].tobytes()
                if x3:
                    want = S.XXH3_64bits(b)
                elif args.workload == "walrec":
                    want = S.crc32c.Mask(S.crc32c.Extend(S.crc32c.Value(bytes([int(tys[k])])), b))
                else:
                    want = S.crc32c.Value(b)
                ok &= int(res[k]) == want
            return ok
        w.check = check
    elif args.workload == "walwrite":
        rng = np.random.default_rng(600 + rank)
        lens = rng.integers(args.wal_len_min, args.wal_len_max + 1, size=args.wal_records).astype(np.uint32)
        offs = np.zeros(len(lens), dtype=np.uint64)
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        src = W.rand_bytes(int(lens.sum()) + 64, dev, 601 + rank)
        frags, nf, nbytes, _ = S.wal_plan(offs, lens, 0, False)
        d_frags = torch.frombuffer(bytearray(bytes(frags)), dtype=torch.uint8).to(dev)
        crc = torch.empty(nf, dtype=torch.int32, device=dev)
        out = torch.zeros(nbytes + 64, dtype=torch.uint8, device=dev)
        from speedb_amd import _lib

        def step():
            _lib.check(_lib.lib.mck_wal_write_batch(src.data_ptr(), d_frags.data_ptr(), nf, 7, crc.data_ptr(),
                                                    out.data_ptr(), stream.cuda_stream), "mck_wal_write_batch")
        w.step = step
        w.launches = 1
        w.span_bytes = int(lens.sum())
        # the one-pass writer k_wal_write_il, one launch per group commit
        # (round 4; workgroups walk their ranges in LDS windows); it reads the
        # payload and the 24 B descriptor once, writes the stream and the 4 B CRC
        w.kernel = "mck::k_wal_write_il (1 launch(es) per step, timed as the step)"
        w.alg_bytes = int(lens.sum()) + nbytes + nf * (24 + 4)
        w.desc = (f"device WAL writer: group commit of {len(lens)} records of "
                  f"{args.wal_len_min}-{args.wal_len_max} B per GPU "
                  f"(README 1 KB values) -> {nf} physical records, {nbytes} B of log stream "
                  "(log::Writer::AddRecord + EmitPhysicalRecord, SURVEY.md 8f row 3)")
        w.cfg = {"records_per_gpu": len(lens), "fragments": nf, "stream_bytes": nbytes}

        def check():
            # the device's log stream walks back to the same records, and
            # every physical record's CRC verifies on the device reader
            step()
            res = S.wal_verify_batch(out, nbytes, 7).cpu().numpy()
            return bool((res[:, 1] == 0).all() and int(res[:, 0].sum()) == nf)
        w.check = check
    elif args.workload == "blob":
        n, kb, vb = args.blob_records, 16, 4096
        rec = 32 + kb + vb
        nbytes = 30 + n * rec
        img = W.rand_bytes(nbytes + 64, dev, 700 + rank)
        recs = img[30:30 + n * rec].view(n, rec)
        recs[:, 0:8] = torch.tensor(list(kb.to_bytes(8, "little")), dtype=torch.uint8, device=dev)
        recs[:, 8:16] = torch.tensor(list(vb.to_bytes(8, "little")), dtype=torch.uint8, device=dev)
        offs = 30 + torch.arange(n, dtype=torch.int64, device=dev) * rec
        lens = torch.full((n,), kb + vb, dtype=torch.int32, device=dev)
        S.blob.WriteRecordCrcs(img, offs, lens)  # BlobLogRecord::EncodeHeaderTo on the device
        status = torch.empty(n, dtype=torch.uint8, device=dev)

        def step():
            S.blob.record_batch(False, img, offs, lens, status=status, stream=stream)
        w.step = step
        w.kernel = _ragged("mck::OpBlobRecord<false>", 4112)
        w.span_bytes = n * rec
        w.alg_bytes = n * (rec + 8 + 4 + 1)
        w.desc = (f"blob file verify: {n} records per GPU ({kb} B key, {vb} B value), header CRC + blob CRC "
                  "of every record (BlobLogRecord::DecodeHeaderFrom + CheckBlobCRC, SURVEY.md 8f row 3)")
        w.cfg = {"records_per_gpu": n, "key_bytes": kb, "value_bytes": vb}

        def check():
            step()
            return int(status.sum().item()) == 0
        w.check = check
    elif args.workload == "kv":
        count, kb, vb = args.kvs, 16, args.kv_value_bytes
        keys = W.rand_bytes(count * kb + 64, dev, 400 + rank)
        vals = W.rand_bytes(count * vb + 64, dev, 401 + rank)
        ks, vs = S.Spans.uniform(keys, kb, count), S.Spans.uniform(vals, vb, count)
        ops = W.rand_bytes(count, dev, 402 + rank)
        seqs = torch.arange(count, dtype=torch.int64, device=dev) + (rank << 40)
        out = torch.empty(count, dtype=torch.int64, device=dev)
        w.step = lambda: S.kv_protect_batch(S.ProtectionKind.KVOS, ks, vs, ops, seqs, out=out, stream=stream)
        w.kernel = ("mck::k_xph3_quads<mck::OpKvProtect<false> >" if vb <= 240
                    else "mck::k_xph3<mck::OpKvProtect<false> >")
        w.span_bytes = count * (kb + vb)
        w.alg_bytes = count * (kb + vb + 1 + 8 + 8)
        w.desc = (f"per-KV protection ProtectKVO(key, value, op).ProtectS(seqno) (db/kv_checksum.h) of "
                  f"{count} KVs per GPU, {kb} B keys + {vb} B values"
                  + (" (README 80M-key/1KB-value shape)" if vb == 1000 else ""))
        w.cfg = {"kvs_per_gpu": count, "key_bytes": kb, "value_bytes": vb}

        def check():
            # the batched kernel == ProtectionInfo64 composed from scalar
            # NPHash64 field hashes (both on the GPU, different code paths)
            import random
            res = out.cpu().numpy().view(np.uint64)
            kh = keys.cpu().numpy()
            vh = vals.cpu().numpy()
            oh = ops.cpu().numpy()
            ok = True
            for i in random.Random(rank).sample(range(count), 16):
                k = kh[i * kb:(i + 1) * kb].tobytes()
                v = vh[i * vb:(i + 1) * vb].tobytes()
                want = (S.NPHash64(k, 0) ^ S.NPHash64(v, 0xD28AAD72F49BD50B)
                        ^ S.NPHash64(bytes([int(oh[i])]), 0xA5155AE5E937AA16)
                        ^ S.NPHash64(int(i + (rank << 40)).to_bytes(8, "little"), 0x77A00858DDD37F21))
                ok &= int(res[i]) == want
            return ok
        w.check = check
    elif args.workload == "blockkv":
        from speedb_amd import _lib
        L = _lib.lib
        db = W.DataBlocks(args.blocks, dev, value_bytes=args.kv_value_bytes, seed=30 + rank)
        n, pb = db.count, args.kv_prot_bytes
        kbase = torch.empty(n + 1, dtype=torch.int64, device=dev)
        abase = torch.empty(n + 1, dtype=torch.int64, device=dev)
        status = torch.empty(n, dtype=torch.int32, device=dev)
        rint = torch.empty(n, dtype=torch.int32, device=dev)
        scratch = torch.empty(int(L.mck_block_kv_scratch_bytes(n)), dtype=torch.uint8, device=dev)
        nkeys = int(db.keys_per_block.sum())
        kbytes = sum(len(k) for e in db.entries for k, _ in e) * (n // db.distinct) + sum(
            len(k) for e in db.entries[:n % db.distinct] for k, _ in e)
        sp = db.spans.c()
        if args.kv_two_pass:
            work = torch.empty(int(L.mck_block_kv_work_bytes(nkeys, kbytes)), dtype=torch.uint8, device=dev)
            out = torch.empty(nkeys * pb, dtype=torch.uint8, device=dev)
            tot = torch.empty(2, dtype=torch.int64, pin_memory=True)

            def step():
                _lib.check(L.mck_block_kv_layout_batch(0, ctypes.byref(sp), kbase.data_ptr(), abase.data_ptr(),
                                                       rint.data_ptr(),
                                                       status.data_ptr(), scratch.data_ptr(), stream.cuda_stream),
                           "mck_block_kv_layout_batch")
                # the totals size the work area: one 16-byte readback per batch
                tot[0].copy_(kbase[n], non_blocking=True)
                tot[1].copy_(abase[n], non_blocking=True)
                stream.synchronize()
                assert int(tot[0]) == nkeys and int(tot[1]) == kbytes
                _lib.check(L.mck_block_kv_protect_batch(0, ctypes.byref(sp), pb, kbase.data_ptr(), abase.data_ptr(),
                                                        rint.data_ptr(), nkeys, work.data_ptr(), out.data_ptr(),
                                                        stream.cuda_stream),
                           "mck_block_kv_protect_batch")
            w.kernel = ("k_block_layout_t + k_blk_scan + k_block_kv_t + k_block_long_rows "
                        "(whole step, incl. the totals readback)")
        else:
            # one pass: slots sized to the batch's largest block (entries)
            slot_cap = int(db.keys_per_block.max())
            work = torch.empty(int(L.mck_block_kv_blocks_work_bytes(n, slot_cap, 0)), dtype=torch.uint8, device=dev)
            out = torch.empty(n * slot_cap * pb, dtype=torch.uint8, device=dev)

            def step():
                _lib.check(L.mck_block_kv_protect_blocks_batch(0, ctypes.byref(sp), pb, slot_cap, 0, kbase.data_ptr(),
                                                               abase.data_ptr(), rint.data_ptr(), status.data_ptr(),
                                                               work.data_ptr(), out.data_ptr(), stream.cuda_stream),
                           "mck_block_kv_protect_blocks_batch")
            w.kernel = ("k_block_kv_walk + k_blk_scan + k_block_kv_flush + k_block_long_rows "
                        "(whole step: mck_block_kv_protect_blocks_batch)")
        w.step = step
        w.span_bytes = db.block_bytes
        # what the step must move: every block read once, the kv_checksum
        # array written (+ 8 B offset, 4 B length per block in, 8 B key base
        # + 4 B status out)
        w.alg_bytes = db.block_bytes + nkeys * pb + n * (8 + 4 + 8 + 4)
        w.kern_from_wall = True
        w.desc = (f"per-KV protection of {n} uncompressed data blocks per GPU (~4 KiB, BlockBuilder layout, "
                  f"restart interval 16, {len(db.entries[0][0][0])} B internal keys, {args.kv_value_bytes} B "
                  f"values, {nkeys} entries), protection_bytes_per_key {pb}: "
                  "Block::InitializeDataBlockProtectionInfo (SURVEY.md 8f row 4)")
        w.cfg = {"blocks_per_gpu": n, "entries": nkeys, "value_bytes": args.kv_value_bytes, "prot_bytes": pb,
                 "path": "two-pass" if args.kv_two_pass else "one-pass"}

        def check():
            # sampled entries == ProtectKV composed from scalar NPHash64 calls
            # (the engine's scalar path, a different kernel)
            import random
            kb = kbase.cpu().numpy()
            ck = out.cpu().numpy()
            ok = bool((status == 0).all().item())
            for i in random.Random(rank).sample(range(n), 8):
                ents = db.entries[i % db.distinct]
                for e in sorted({0, 1, 2, len(ents) - 2, len(ents) - 1} & set(range(len(ents)))):
                    k, v = ents[e]
                    want = S.NPHash64(k, 0) ^ S.NPHash64(v, 0xD28AAD72F49BD50B)
                    got = ck[(kb[i] + e) * pb:(kb[i] + e + 1) * pb].tobytes()
                    ok &= got == (want & (2 ** (8 * pb) - 1)).to_bytes(pb, "little")
            return ok
        w.check = check
    else:  # host
        from speedb_amd import _lib
        # configs[4]: the 80M-key / 1 KB-value compaction stream cut into
        # SST-sized blocks (4 x (16 B key + 1000 B value) + overhead = 4300 B,
        # FlushBlockBySizePolicy), 8-GPU share per GPU, in pinned host memory
        block = 4300
        count = args.host_blocks
        ndev = args.host_ndev
        if ndev > 0 and (world > 1 or ndev > torch.cuda.device_count()):
            raise SystemExit(f"bench: --host-ndev {ndev} needs one process and {ndev} visible GPU(s) "
                             f"(world {world}, {torch.cuda.device_count()} visible)")
        count *= max(1, ndev)  # configs[4]'s per-GPU share for each device
        hbuf = torch.empty(count * block + 64, dtype=torch.uint8, pin_memory=True)
        tile = torch.randint(0, 256, (256 << 20,), dtype=torch.uint8, generator=torch.Generator().manual_seed(5))
        for o in range(0, hbuf.numel(), tile.numel()):  # 256 MiB of random bytes, tiled
            n = min(tile.numel(), hbuf.numel() - o)
            hbuf[o:o + n].copy_(tile[:n])
        out = np.empty(count, dtype=np.uint32)
        secs = ctypes.c_double()

        def step():
            _lib.check(_lib.lib.mck_host_batch_checksum(
                1, hbuf.data_ptr(), None, None, block, block, count, 0, ndev, 256 << 20,
                out.ctypes.data, None, ctypes.byref(secs)), "mck_host_batch_checksum")
        w.step = step
        w.kernel = _ragged("mck::OpCrcValueZ", 4300) + " (H2D/D2H overlapped)"
        w.span_bytes = count * block
        w.alg_bytes = count * (block + 4 + 8 + 4)
        per = count // max(1, ndev)
        w.desc = (f"host-resident pinned {per} x {block} B blocks per GPU (the 8-GPU share of the "
                  "80M-key/1KB-value README stream, SST-sized blocks) -> H2D + CRC32C + D2H, 256 MiB "
                  "double-buffered chunks, copy-inclusive (BASELINE.json configs[4])"
                  + (f"; one process driving {ndev} GPUs" if ndev > 0 else ""))
        w.cfg = {"blocks_per_gpu": per, "block_bytes": block, "pcie_inclusive": True}
        if ndev > 0:
            w.cfg["host_ndev"] = ndev

        def device_only():
            # the same blocks already in HBM (a 4 GiB slice): kernel-only rate
            n = min(count, (4 << 30) // block)
            d = hbuf[:n * block + 64].to(dev)
            sp = S.Spans.uniform(d, block, n)
            res = torch.empty(n, dtype=torch.int32, device=dev)
            for _ in range(20):
                S.crc32c_batch(sp, out=res, stream=stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(20):
                S.crc32c_batch(sp, out=res, stream=stream)
            e1.record(stream)
            torch.cuda.synchronize(dev)
            ms = e0.elapsed_time(e1) / 20
            ok = bool((res.cpu().numpy().view(np.uint32) == out[:n]).all())
            return {"value": round(n * block / (ms * 1e-3) / 2**30, 2), "unit": "GiB/s",
                    "blocks": n, "kernel_ms": round(ms, 4), "agrees_with_host_path": ok}

        def h2d_only():
            # the PCIe leg alone: the same pinned bytes copied H2D in the
            # pipeline's 256 MiB chunks, two device buffers alternating
            chunk = 256 << 20
            bufs = [torch.empty(chunk, dtype=torch.uint8, device=dev) for _ in range(2)]
            tot = count * block
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for k, o in enumerate(range(0, tot, chunk)):
                n = min(chunk, tot - o)
                bufs[k & 1][:n].copy_(hbuf[o:o + n], non_blocking=True)
            torch.cuda.synchronize(dev)
            dt = time.perf_counter() - t0
            del bufs
            return {"GBps": round(tot / dt / 1e9, 2), "GiBps": round(tot / dt / 2**30, 2), "seconds": round(dt, 4)}

        def check():
            # host-pipeline results == the device-resident kernel's on the
            # same blocks (all of the 4 GiB slice), and its rate; the H2D
            # copy alone for the overlap figure
            w.device_only = device_only()
            w.h2d_only = h2d_only()
            return w.device_only["agrees_with_host_path"]
        w.check = check
    return w


def shim_latency(args):
    """Per-call latency of the synchronous scalar shim vs the CPU reference
    (INTEGRATION.md keeps crc32c::Extend on the CPU below the crossover)."""
    import numpy as np
    import torch

    from speedb_amd import _lib
    torch.cuda.set_device(0)
    L = _lib.lib
    ref = None
    p = os.path.join(REPO, "oracle", "_ref", "libspdb_ref.so")
    if os.path.exists(p):
        ref = ctypes.CDLL(p)
        ref.ref_crc32c_value.restype = ctypes.c_uint32
        ref.ref_crc32c_value.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    rows = []
    out = ctypes.c_uint32()
    for n in (64, 4096, 32768, 1 << 20, 16 << 20):
        buf = np.random.default_rng(n).integers(0, 256, size=n, dtype=np.uint8)
        ptr = buf.ctypes.data
        for _ in range(20):
            _lib.check(L.mck_crc32c_value_r(ptr, n, ctypes.byref(out)), "mck_crc32c_value_r")
        reps = max(20, min(2000, int(2e8 // max(n, 1))))
        t0 = time.perf_counter()
        for _ in range(reps):
            L.mck_crc32c_value_r(ptr, n, ctypes.byref(out))
        gpu_us = (time.perf_counter() - t0) / reps * 1e6
        row = {"bytes": n, "shim_us": round(gpu_us, 2)}
        if ref is not None:
            assert ref.ref_crc32c_value(ptr, n) == out.value
            r2 = max(reps, 200)
            t0 = time.perf_counter()
            for _ in range(r2):
                ref.ref_crc32c_value(ptr, n)
            cpu_us = (time.perf_counter() - t0) / r2 * 1e6
            row["cpu_reference_us"] = round(cpu_us, 3)
        rows.append(row)
    print(json.dumps({"metric": "scalar shim latency (mck_crc32c_value_r, pageable host buffer, sync)",
                      "unit": "us per call", "rows": rows,
                      "note": "cpu_reference_us = crc32c::Value from oracle/_ref on one host thread, "
                              "including the ctypes call overhead (~0.3 us)"}))


def batch_latency(args):
    """Latency of ONE small VerifyBlockChecksum batch -- the RetrieveMultipleBlocks
    shape (table/block_based/block_based_table_reader_sync_and_async.h
    :217-228: at most 32 blocks of a MultiGet, read together and verified one
    by one) -- against the reference verifying the same blocks on the calling
    thread.  Blocks: 4096 + 0..255 B payload + 5-byte trailer (kCRC32c,
    FlushBlockBySizePolicy sizes).  Per batch of n blocks:
      device_us -- blocks already in HBM: mck_sst_verify_batch + stream sync;
      pinned_us -- blocks in pinned host memory: H2D of the blocks and their
                   descriptors, the verify, D2H of the n mismatch flags, sync;
      cpu_us    -- the reference's crc32c::Value over the n blocks on one
                   host thread (oracle/_ref, cache-hot: the blocks were just
                   read), what VerifyBlockChecksum costs per block."""
    import random

    import numpy as np
    import torch

    import speedb_amd as S
    from speedb_amd import _lib
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    L = _lib.lib
    ref = None
    p = os.path.join(REPO, "oracle", "_ref", "libspdb_ref.so")
    if os.path.exists(p):
        ref = ctypes.CDLL(p)
        ref.ref_bench.restype = ctypes.c_uint64
        ref.ref_bench.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_uint64,
                                  ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                  ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint32)]
    rows = []
    rnd = random.Random(1)
    for n in (1, 8, 32, 256):
        lens = [4096 + rnd.randrange(0, 256) for _ in range(n)]
        offs, pos = [], 0
        for ln in lens:
            offs.append(pos)
            pos += ln + 5
        img = bytearray(np.random.default_rng(n).integers(0, 256, size=pos + 64, dtype=np.uint8).tobytes())
        for o, ln in zip(offs, lens):  # seal every block (type 0, kCRC32c, no context)
            img[o + ln] = 0
            struct_v = S.crc32c.Mask(S.crc32c.Value(bytes(img[o:o + ln + 1])))
            img[o + ln + 1:o + ln + 5] = struct_v.to_bytes(4, "little")
        nb = len(img)
        desc = np.zeros(n * 3, dtype=np.uint32)  # [offsets as 2 x u32][lengths]
        desc[:2 * n] = np.array(offs, dtype=np.uint64).view(np.uint32)
        desc[2 * n:] = lens
        h_img = torch.frombuffer(img, dtype=torch.uint8).pin_memory()
        h_desc = torch.from_numpy(desc.view(np.uint8)).pin_memory()
        d_img = torch.empty(nb, dtype=torch.uint8, device=dev)
        d_desc = torch.empty(h_desc.numel(), dtype=torch.uint8, device=dev)
        d_mm = torch.empty(n, dtype=torch.uint8, device=dev)
        h_mm = torch.empty(n, dtype=torch.uint8).pin_memory()
        d_img.copy_(h_img)
        d_desc.copy_(h_desc)
        torch.cuda.synchronize()
        sp = _lib.mck_spans(d_img.data_ptr(), d_desc.data_ptr(), d_desc.data_ptr() + 8 * n, 0, 0, n)
        sst = st.cuda_stream

        def verify():
            _lib.check(L.mck_sst_verify_batch(1, ctypes.byref(sp), None, 0, d_mm.data_ptr(), None, None, None, sst),
                       "mck_sst_verify_batch")

        def timed(fn, reps):
            for _ in range(50):
                fn()
            st.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                fn()
            return (time.perf_counter() - t0) / reps * 1e6

        def dev_call():
            verify()
            st.synchronize()

        def pinned_call():
            d_img.copy_(h_img, non_blocking=True)
            d_desc.copy_(h_desc, non_blocking=True)
            verify()
            h_mm.copy_(d_mm, non_blocking=True)
            st.synchronize()

        dev_us = timed(dev_call, 2000)
        pin_us = timed(pinned_call, 2000)
        assert int(h_mm.sum()) == 0
        row = {"blocks": n, "bytes": sum(lens), "device_us": round(dev_us, 2), "pinned_us": round(pin_us, 2)}
        if ref is not None:
            # the reference on one thread over the same n blocks (uniform
            # 4224-B blocks: the mean of these sizes), cache-hot
            blk = 4224
            buf = np.frombuffer(bytes(img[:max(nb, n * blk)]) + bytes(max(0, n * blk - nb)), dtype=np.uint8)
            secs, sink = ctypes.c_double(), ctypes.c_uint32()
            passes = max(1, 200000 // n)
            tot = ref.ref_bench(0, 1, 1, blk, 0, buf.ctypes.data, n, passes, ctypes.byref(secs), ctypes.byref(sink))
            row["cpu_us"] = round(secs.value / passes * 1e6, 3)
            row["cpu_GiBps"] = round(tot / secs.value / 2**30, 2)
        rows.append(row)
    cross_dev = next((r["blocks"] for r in rows if "cpu_us" in r and r["device_us"] < r["cpu_us"]), None)
    cross_pin = next((r["blocks"] for r in rows if "cpu_us" in r and r["pinned_us"] < r["cpu_us"]), None)
    print(json.dumps({"metric": "latency of one small VerifyBlockChecksum batch (RetrieveMultipleBlocks shape)",
                      "unit": "us per batch", "rows": rows,
                      "crossover_blocks_device_resident": cross_dev, "crossover_blocks_pinned": cross_pin,
                      "note": "device_us/pinned_us include the launch and a stream synchronize; cpu_us = "
                              "crc32c::Value of oracle/_ref over the same number of ~4.2 KiB blocks on one "
                              "host thread"}))


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(argv, nprocs: int, script: str = None, env=None) -> int:
    """Start `nprocs` fresh ranks of `script` (default: this file) with
    torch.distributed.run on this node and return its exit code.  A child
    process, never an exec: the caller has not touched the GPU (counting
    devices does not), and on this pool exec'ing a process that has is
    fatal."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nprocs}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", script or os.path.abspath(__file__)]
    return subprocess.call(cmd + list(argv), env=env)


def check_world(requested, world_env) -> int:
    """The ranks this process belongs to: WORLD_SIZE when launched by
    torchrun (which --gpus, if given, must equal), else 1."""
    world = int(world_env) if world_env else 1
    if requested is not None and requested != world:
        raise SystemExit(f"bench: --gpus {requested} but WORLD_SIZE={world}")
    return world


def main():
    args = parse()
    if args.engine_lib:  # the only way a bench run loads another engine build (speedb_amd/_lib.py)
        os.environ["SPEEDB_AMD_LIB"] = os.path.abspath(args.engine_lib)
        os.environ["SPEEDB_AMD_AB"] = "1"
    if args.workload == "shim":
        return shim_latency(args)
    if args.workload == "latency":
        return batch_latency(args)
    import torch
    import torch.distributed as dist

    if "WORLD_SIZE" not in os.environ and (args.gpus or 1) > 1:
        # --gpus N from a plain `python bench.py`: N ranks, one per GPU, started
        # here (device_count does not initialise the GPU on this image)
        have = torch.cuda.device_count()
        if args.gpus > have:
            print(f"bench: --gpus {args.gpus} but only {have} GPU(s) visible", file=sys.stderr)
            return 2
        return launch_ranks(sys.argv[1:], args.gpus)
    world = check_world(args.gpus, os.environ.get("WORLD_SIZE"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if local >= torch.cuda.device_count():
        print(f"bench: rank {rank} has local rank {local} but {torch.cuda.device_count()} GPU(s)", file=sys.stderr)
        return 2
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
        assert dist.get_world_size() == world, (dist.get_world_size(), world)

    from speedb_amd import _lib, shard
    if args.crc_driver != "auto" or args.crc_order != "blocked":
        drv = {"auto": 0, "rows16": 2, "rows8": 3, "rows4": 5, "rows1": 6, "bh": 7}[args.crc_driver]
        _lib.check(_lib.lib.mck_test_set_crc_driver(drv, 1 if args.crc_order == "interleaved" else 0),
                   "mck_test_set_crc_driver")
    w = make_workload(args, dev, rank, world)
    stream = torch.cuda.current_stream(dev)
    # clock settle: untimed work for --settle-ms, then the W warmup steps
    t_settle = time.perf_counter()
    while (time.perf_counter() - t_settle) * 1e3 < args.settle_ms:
        for _ in range(4):
            w.step()
        torch.cuda.synchronize(dev)
    for _ in range(args.warmup):
        w.step()
    torch.cuda.synchronize(dev)
    shard.barrier(dev)
    torch.cuda.synchronize(dev)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        w.step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    shard.barrier(dev)
    torch.cuda.synchronize(dev)
    wall = shard.reduce_max(time.perf_counter() - t0, dev)
    kern_ms = ev0.elapsed_time(ev1) / (args.steps * w.launches) / getattr(w, "kern_scale", 1.0)
    if getattr(w, "kern_from_wall", False):  # a step with a host sync inside: the step is the unit
        kern_ms = wall / args.steps * 1e3

    verified = None if args.no_verify else w.check()
    if verified is False:
        print("bench: RESULT CHECK FAILED", file=sys.stderr)

    value = shard.reduce_sum(int(w.span_bytes), dev) * args.steps / wall / 2**30
    roof = None
    if args.workload != "host":
        achieved = w.alg_bytes / (kern_ms * 1e-3)
        roof = {
            "bound": "hbm", "achieved": round(achieved / 1e9, 1), "peak": HBM_PEAK / 1e9,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK, 4), "traffic": None,
            "kernel": w.kernel, "kernel_avg_ms": round(kern_ms, 4),
            "alg_bytes_per_launch": int(w.alg_bytes),
        }
        # the tracked PMC traffic of this exact workload, config and kernel
        # (profiles/traffic_*.json, one file per profiled shape)
        import glob
        for tf in sorted(glob.glob(os.path.join(REPO, "profiles", "traffic_*.json"))):
            with open(tf) as f:
                tr = json.load(f)
            if (tr.get("workload", args.workload) == args.workload and tr.get("config") == w.cfg
                    and tr.get("kernel") == w.kernel):
                roof["traffic"] = tr["hbm_bytes_per_launch"]
                roof["traffic_source"] = os.path.relpath(tf, REPO)
                break
    cpu = None
    if (rank == 0 and world == 1 and args.cpu_seconds > 0 and not args.no_verify
            and args.workload in ("crc32c", "xxh3")):
        cpu = cpu_baseline(args, args.workload, args.block_bytes, w.sample, w.results)
        if cpu is not None:
            verified = cpu["agrees_with_gpu"]
            if not verified:
                print("bench: GPU checksums disagree with the reference", file=sys.stderr)
    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "GiB/s",
            "n_gpus": dist.get_world_size() if world > 1 else world * max(1, args.host_ndev),
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(wall / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": getattr(w, "scaling", "weak"), "vs_baseline": None, "dtype": "u8",
            "data": "synthetic: random bytes generated on-device (device-resident)"
                    if args.workload != "host" else "synthetic: random bytes in pinned host memory",
            "config": dict({"workload": w.desc, "parallelism": f"partitioned x{world} (no collective)"},
                           **w.cfg),
            "roofline": roof, "cpu_baseline": cpu, "verified": verified,
            "engine": _lib.lib_identity(),
        }
        if getattr(w, "device_only", None):
            line["device_only"] = w.device_only
        if getattr(w, "h2d_only", None) and args.host_ndev <= 0:
            # the copy-inclusive step against its PCIe leg alone: what the
            # kernels, the D2H of the results and the pipeline's fill and
            # drain add on top of the H2D copy
            t_step = wall / args.steps
            t_h2d = w.h2d_only["seconds"]
            t_kern = w.span_bytes / (w.device_only["value"] * 2**30)
            line["h2d_only"] = dict(w.h2d_only, copy_inclusive_over_h2d=round(t_h2d / t_step, 4),
                                    excess_over_h2d_ms=round((t_step - t_h2d) * 1e3, 2),
                                    kernel_ms_at_device_rate=round(t_kern * 1e3, 2))
        if getattr(w, "end_to_end", None):
            line["end_to_end"] = w.end_to_end
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)

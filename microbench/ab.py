#!/usr/bin/env python3
"""Interleaved same-process A/B timing of engine builds (design tool).

usage: python microbench/ab.py lib1.so lib2.so ... [--blocks N] [--block B]
       [--rounds R] [--iters K] [--kind crc32c|xxh3] [--mixed]

Every variant runs K launches per round, rounds interleaved, on the same
device-resident data; prints median / min kernel time and TB/s per variant
and checks that all variants produce identical results.
"""
import argparse
import ctypes
import statistics
import sys

import torch


class Spans(ctypes.Structure):
    _fields_ = [("base", ctypes.c_void_p), ("offsets", ctypes.c_void_p),
                ("lengths", ctypes.c_void_p), ("stride", ctypes.c_uint64),
                ("length", ctypes.c_uint32), ("count", ctypes.c_uint32)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--blocks", type=int, default=1 << 20)
    ap.add_argument("--block", type=int, default=4096)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--kind", default="crc32c", help="crc32c | xxh3 | wal")
    ap.add_argument("--mixed", action="store_true",
                    help="compaction-shaped 4/16/64 KiB (+0..255) spans at odd offsets")
    ap.add_argument("--align", type=int, default=1,
                    help="--mixed: round every span start up to this many bytes")
    ap.add_argument("--nojitter", action="store_true", help="--mixed: no +0..255 length jitter")
    ap.add_argument("--ragged", action="store_true",
                    help="uniform blocks passed with explicit offsets/lengths (the generic driver)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    if a.kind == "wal":
        # a.blocks WAL blocks of 32 KiB, one kFullType record each; record
        # CRCs written by the first library
        count = a.blocks
        data = torch.randint(0, 256, (count * 32768 + 64,), dtype=torch.uint8, device=dev, generator=g)
        pay = Spans(data.data_ptr() + 7, None, None, 32768, 32761, count)
        span_bytes = count * 32768
    elif a.mixed:
        import random
        rnd = random.Random(3)
        lens, offs, pos = [], [], 0
        total = a.blocks * a.block
        while pos < total:
            n = rnd.choice([4096] * 6 + [16384] * 3 + [65536]) + rnd.randrange(0, 256)
            if a.nojitter:
                n &= ~255
            pos = (pos + a.align - 1) // a.align * a.align
            offs.append(pos)
            lens.append(n)
            pos += n + 5
        nbytes = pos + 64
        count = len(lens)
        o = torch.tensor(offs, dtype=torch.int64, device=dev)
        l_ = torch.tensor(lens, dtype=torch.int32, device=dev)
        data = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device=dev, generator=g)
        sp = Spans(data.data_ptr(), o.data_ptr(), l_.data_ptr(), 0, 0, count)
        span_bytes = sum(lens)
    else:
        count = a.blocks
        data = torch.randint(0, 256, (count * a.block + 64,), dtype=torch.uint8, device=dev, generator=g)
        sp = Spans(data.data_ptr(), None, None, a.block, a.block, count)
        if a.ragged:
            o = torch.arange(count, dtype=torch.int64, device=dev) * a.block
            l_ = torch.full((count,), a.block, dtype=torch.int32, device=dev)
            sp = Spans(data.data_ptr(), o.data_ptr(), l_.data_ptr(), 0, 0, count)
        span_bytes = count * a.block
    libs = []
    for p in a.libs:
        L = ctypes.CDLL(p)
        L.mck_crc32c_batch.argtypes = [ctypes.POINTER(Spans), ctypes.c_void_p, ctypes.c_uint32,
                                       ctypes.c_void_p, ctypes.c_void_p]
        L.mck_xxh3_64_batch.argtypes = [ctypes.POINTER(Spans), ctypes.c_void_p, ctypes.c_void_p]
        L.mck_wal_record_crc_batch.argtypes = [ctypes.POINTER(Spans), ctypes.c_void_p, ctypes.c_uint32,
                                               ctypes.c_void_p, ctypes.c_void_p]
        L.mck_wal_verify_batch.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                           ctypes.c_void_p, ctypes.c_void_p]
        libs.append(L)
    if a.kind == "wal":
        types = torch.ones(count, dtype=torch.uint8, device=dev)
        crc = torch.empty(count, dtype=torch.int32, device=dev)
        assert libs[0].mck_wal_record_crc_batch(ctypes.byref(pay), types.data_ptr(), 7, crc.data_ptr(), None) == 0
        blocks = data[:count * 32768].view(count, 32768)
        blocks[:, 0:4] = crc.view(torch.uint8).view(count, 4)
        blocks[:, 4] = 32761 & 0xFF
        blocks[:, 5] = 32761 >> 8
        blocks[:, 6] = 1
        torch.cuda.synchronize()
    stream = torch.cuda.current_stream(dev)
    outs = []
    for L in libs:
        if a.kind == "wal":
            out = torch.zeros((count, 4), dtype=torch.int32, device=dev)
            f = (lambda L=L, out=out: L.mck_wal_verify_batch(data.data_ptr(), count * 32768, 7, out.data_ptr(),
                                                             stream.cuda_stream))
        elif a.kind == "crc32c":
            out = torch.zeros(count, dtype=torch.int32, device=dev)
            f = (lambda L=L, out=out: L.mck_crc32c_batch(ctypes.byref(sp), None, 0, out.data_ptr(),
                                                         stream.cuda_stream))
        else:
            out = torch.zeros(count, dtype=torch.int64, device=dev)
            f = (lambda L=L, out=out: L.mck_xxh3_64_batch(ctypes.byref(sp), out.data_ptr(),
                                                          stream.cuda_stream))
        assert f() == 0
        outs.append((f, out))
    torch.cuda.synchronize()
    for i in range(1, len(outs)):
        same = torch.equal(outs[0][1], outs[i][1])
        print(f"variant {i} results identical to variant 0: {same}")
        if not same:
            sys.exit(1)
    times = [[] for _ in libs]
    for _ in range(a.rounds):
        for v, (f, _) in enumerate(outs):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(a.iters):
                f()
            e1.record(stream)
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / a.iters)
    for p, t in zip(a.libs, times):
        med = statistics.median(t)
        print(f"{p:40s} median {med:.4f} ms  min {min(t):.4f} ms  "
              f"{span_bytes / med / 1e9:.3f} TB/s  ({span_bytes / med / 1e9 / 8.0 * 100:.1f}% of 8 TB/s)")


if __name__ == "__main__":
    main()

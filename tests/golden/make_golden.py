#!/usr/bin/env python3
"""Regenerate the golden fixtures in tests/golden/ from the REFERENCE.

Runs in the build container only: it loads oracle/_ref/libspdb_ref.so, the
reference's own util/crc32c.cc + util/xxhash.cc compiled in place by
oracle/Makefile (nothing of the reference is copied here), and records its
outputs on seeded inputs.  The committed fixtures are data: an input blob and
the reference's outputs.

  blob.bin       128 KiB of splitmix64 bytes (seed 0x5eedb10c), see blob_bytes()
  vectors.json   per-case reference outputs over slices of blob.bin, plus the
                 block-trailer / WAL-record cases and ChecksumModifierForContext
                 cases from the reference's own inline table/format.h
  kat.json       known-answer values quoted from the reference's own tests
                 (util/crc32c_test.cc, table/table_test.cc)

usage: python tests/golden/make_golden.py
"""
import ctypes
import json
import os
import random
import struct

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_SO = os.path.join(REPO, "oracle", "_ref", "libspdb_ref.so")

BLOB_SEED = 0x5EEDB10C
BLOB_BYTES = 128 * 1024
M64 = (1 << 64) - 1


def splitmix64_words(seed: int, n: int):
    out = []
    for i in range(n):
        z = (seed + (i + 1) * 0x9E3779B97F4A7C15) & M64
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
        out.append(z ^ (z >> 31))
    return out


def blob_bytes() -> bytes:
    return struct.pack(f"<{BLOB_BYTES // 8}Q", *splitmix64_words(BLOB_SEED, BLOB_BYTES // 8))


def load_ref():
    r = ctypes.CDLL(REF_SO)
    sig = {
        "ref_crc32c_extend": (ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_char_p, ctypes.c_size_t]),
        "ref_crc32c_value": (ctypes.c_uint32, [ctypes.c_char_p, ctypes.c_size_t]),
        "ref_crc32c_mask": (ctypes.c_uint32, [ctypes.c_uint32]),
        "ref_crc32c_combine": (ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_size_t]),
        "ref_xxh3_64": (ctypes.c_uint64, [ctypes.c_char_p, ctypes.c_size_t]),
        "ref_xxh32": (ctypes.c_uint32, [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32]),
        "ref_xxh64": (ctypes.c_uint64, [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint64]),
        "ref_builtin_checksum": (ctypes.c_uint32, [ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t]),
        "ref_wal_record_crc": (ctypes.c_uint32, [ctypes.c_uint8, ctypes.c_char_p, ctypes.c_size_t,
                                                 ctypes.c_int, ctypes.c_uint32]),
        "ref_context_modifier": (ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_uint64]),
        "ref_hash64": (ctypes.c_uint64, [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint64]),
        "ref_kv_protect": (ctypes.c_uint64, [ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p,
                                             ctypes.c_size_t, ctypes.c_uint8, ctypes.c_uint64]),
    }
    for k, (res, args) in sig.items():
        f = getattr(r, k)
        f.restype, f.argtypes = res, args
    return r


def main():
    ref = load_ref()
    blob = blob_bytes()
    with open(os.path.join(HERE, "blob.bin"), "wb") as f:
        f.write(blob)
    rng = random.Random(20261015)
    lengths = (list(range(0, 18)) + [31, 32, 33, 63, 64, 65, 127, 128, 129, 240, 241, 255, 256,
                                     1023, 1024, 1025, 4095, 4096, 4097, 16383, 16384, 16385,
                                     32761, 32762, 65535, 65536, 65537]
               + [rng.randrange(0, 70000) for _ in range(48)])
    cases = []
    for i, n in enumerate(lengths):
        off = i % 8 if i % 3 else rng.randrange(0, 4096)
        off = min(off, BLOB_BYTES - n)
        d = blob[off:off + n]
        init = rng.getrandbits(32)
        c = {
            "off": off, "len": n,
            "crc32c": ref.ref_crc32c_value(d, n),
            "extend_init": init, "crc32c_extend": ref.ref_crc32c_extend(init, d, n),
            "xxh3": ref.ref_xxh3_64(d, n),
            "xxh32": ref.ref_xxh32(d, n, 0),
            "xxh64": ref.ref_xxh64(d, n, 0),
            "builtin": {str(t): ref.ref_builtin_checksum(t, d, n) for t in range(5)},
        }
        # WithLastByte(type, d[:n-1], d[n-1]) == builtin(type, d) (table_test.cc:2297-2300)
        cases.append(c)
    combine = []
    for _ in range(64):
        a, b, n = rng.getrandbits(32), rng.getrandbits(32), rng.choice([0, 1, 3, 4, 5, 1000, 4096, 32761,
                                                                       rng.randrange(0, 1 << 24)])
        combine.append({"crc1": a, "crc2": b, "len2": n, "out": ref.ref_crc32c_combine(a, b, n)})
    ctx = []
    for _ in range(32):
        base = rng.choice([0, rng.getrandbits(32)])
        off = rng.getrandbits(rng.choice([12, 32, 40, 64]))
        ctx.append({"base": base, "offset": off, "out": ref.ref_context_modifier(base, off)})
    # edge offsets (carry out of the low word, 4 GiB multiples, all-ones)
    # from their own generator so the draws of the other fixtures stay put
    rng3 = random.Random(20261017)
    for off in ([0, 1, 0xFFFFFFFF, 1 << 32, (1 << 32) + 1, 0xFFFFFFFFFFFFFFFF, 0x8000000080000000,
                 0xFFFFFFFF00000001] + [rng3.getrandbits(64) for _ in range(24)]):
        for base in (0, 1, 0xFFFFFFFF, rng3.getrandbits(32)):
            ctx.append({"base": base, "offset": off, "out": ref.ref_context_modifier(base, off)})
    wal = []
    for _ in range(40):
        t = rng.choice([1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11])
        n = rng.choice([0, 1, 7, 100, 1000, 32761, rng.randrange(0, 32757)])
        off = rng.randrange(0, BLOB_BYTES - n)
        recyclable = 1 if t in (5, 6, 7, 8, 11) else 0
        ln = rng.choice([123, 0, 0xFFFFFFFF, rng.getrandbits(32)])
        wal.append({"type": t, "off": off, "len": n, "recyclable": recyclable, "log_number": ln,
                    "crc": ref.ref_wal_record_crc(t, blob[off:off + n], n, recyclable, ln)})
    type_crc = [ref.ref_crc32c_value(bytes([t]), 1) for t in range(12)]
    # per-KV protection (db/kv_checksum.h): Hash64 = XXPH3 with the field seeds
    rng2 = random.Random(20261016)
    seeds = [0, 0xD28AAD72F49BD50B, 0xA5155AE5E937AA16, 0x77A00858DDD37F21, 0x4A2AB5CBD26F542C]
    hash64 = []
    for n in (list(range(0, 260)) + [511, 512, 513, 1000, 1023, 1024, 1025, 1088, 2047, 2048, 2049,
                                     3071, 3072, 4096, 4100, 8191, 16384]
              + [rng2.randrange(0, 20000) for _ in range(24)]):
        off = rng2.randrange(0, BLOB_BYTES - n)
        seed = seeds[n % 5] if n % 7 else rng2.getrandbits(64)
        hash64.append({"off": off, "len": n, "seed": seed,
                       "out": ref.ref_hash64(blob[off:off + n], n, seed)})
    kv = []
    for i in range(200):
        kn = rng2.choice([0, 1, 8, 16, 24, rng2.randrange(0, 300)])
        vn = rng2.choice([0, 1, 100, 240, 241, 1000, 1024, rng2.randrange(0, 5000)])
        ko, vo = rng2.randrange(0, BLOB_BYTES - kn), rng2.randrange(0, BLOB_BYTES - vn)
        mode, op, extra = i % 4, rng2.randrange(0, 256), rng2.getrandbits(64)
        kv.append({"mode": mode, "koff": ko, "klen": kn, "voff": vo, "vlen": vn, "op": op, "extra": extra,
                   "out": ref.ref_kv_protect(mode, blob[ko:ko + kn], kn, blob[vo:vo + vn], vn, op, extra)})
    out = {"blob_seed": BLOB_SEED, "blob_bytes": BLOB_BYTES, "cases": cases, "combine": combine,
           "context_modifier": ctx, "wal_records": wal, "wal_type_crc": type_crc,
           "hash64": hash64, "kv_protect": kv}
    with open(os.path.join(HERE, "vectors.json"), "w") as f:
        json.dump(out, f, indent=0)
    print(f"wrote {len(cases)} cases, {len(combine)} combine, {len(ctx)} ctx, {len(wal)} wal, "
          f"{len(hash64)} hash64, {len(kv)} kv_protect")


if __name__ == "__main__":
    main()

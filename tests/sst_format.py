"""Test-side writer of block-based-table (SST) images -- TEST INFRASTRUCTURE.

Restates the on-disk layout BlockBasedTableBuilder produces, so the engine's
host SST reader (speedb_amd/csrc/mck_sst.cc) and the batched GPU verify can
be exercised on real-format files without the reference's storage engine
(which cannot be built here: it needs the reference's cmake build).  Block
checksums come from the CPU oracle (oracle/liboracle.so).  Parity of the
*parser* is therefore against this restatement ("parity unpinned" for the
file layout); the checksums themselves are pinned by the oracle.

Reference layout (speedb-io/speedb):
  BlockBuilder entries + restarts        table/block_based/block_builder.cc:45-230
  value delta encoding of index values   table/format.cc:121-135 IndexValue::EncodeTo,
                                         block_builder.cc Add(key, value, delta_value)
  WriteMaybeCompressedBlock trailer      table/block_based/block_based_table_builder.cc:1304-1358
  Finish(): filter, index, compression   block_based_table_builder.cc:1560-1800
    dict, range del, properties,
    metaindex, footer
  properties (varint64 integer props,    table/meta_blocks.cc:60-130,
    fixed32 index type)                  block_based_table_builder.cc:239
  FooterBuilder::Build                   table/format.cc:239-346
"""
from __future__ import annotations

import random
import struct
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

MAGIC = 0x88E241B785F4CFF7
LEGACY_MAGIC = 0xDB4775248B80FB57
TRAILER = 5


def varint(v: int) -> bytes:
    out = bytearray()
    while v >= 128:
        out.append((v & 127) | 128)
        v >>= 7
    out.append(v)
    return bytes(out)


def varsigned(v: int) -> bytes:  # zigzag, util/coding.h PutVarsignedint64
    return varint(((v << 1) ^ (v >> 63)) & 0xFFFFFFFFFFFFFFFF)


def handle(off: int, size: int) -> bytes:
    return varint(off) + varint(size)


def common_prefix(a: bytes, b: bytes) -> int:
    n = min(len(a), len(b))
    i = 0
    while i < n and a[i] == b[i]:
        i += 1
    return i


def build_block(entries: List[Tuple[bytes, bytes]], restart_interval: int = 16,
                delta_values: Optional[List[Optional[bytes]]] = None, hash_buckets: int = 0,
                bucket_fill: int = 0xFF) -> bytes:
    """BlockBuilder: entries (key, value).  With delta_values (index value
    delta encoding, format_version >= 4) there is no value_length field and
    an entry with shared != 0 stores delta_values[i] instead of its value.
    hash_buckets > 0 appends a data-block hash index of that many buckets
    (data_block_hash_index.cc DataBlockHashIndexBuilder::Finish: bucket
    bytes + NUM_BUCK u16) and sets the footer's index-type bit
    (data_block_footer.cc:24-39)."""
    buf = bytearray()
    restarts = []
    last = b""
    for i, (k, v) in enumerate(entries):
        if i % restart_interval == 0:
            restarts.append(len(buf))
            shared = 0
        else:
            shared = common_prefix(last, k)
        buf += varint(shared) + varint(len(k) - shared)
        if delta_values is None:
            buf += varint(len(v)) + k[shared:] + v
        else:
            dv = delta_values[i] if shared != 0 else None
            buf += k[shared:] + (dv if dv is not None else v)
        last = k
    if not restarts:
        restarts = [0]
    for r in restarts:
        buf += struct.pack("<I", r)
    footer = len(restarts)
    if hash_buckets:
        buf += bytes([bucket_fill]) * hash_buckets + struct.pack("<H", hash_buckets)
        footer |= 1 << 31
    buf += struct.pack("<I", footer)
    return bytes(buf)


@dataclass
class Layout:
    """Where the writer put every block (for the parser's expected list)."""
    blocks: List[Tuple[int, int, str]] = field(default_factory=list)  # (offset, size, kind)
    footer_offset: int = 0


class SstWriter:
    """Appends blocks with trailers; `oracle` supplies the builtin checksums."""

    def __init__(self, oracle, checksum_type: int = 1, format_version: int = 5,
                 base_context_checksum: int = 0):
        self.o = oracle
        self.t = checksum_type
        self.fv = format_version
        self.base = base_context_checksum if format_version >= 6 else 0
        self.buf = bytearray()
        self.layout = Layout()

    def write_block(self, payload: bytes, kind: str, comp_type: int = 0) -> Tuple[int, int]:
        off = len(self.buf)
        ck = self.o.BuiltinLast(self.t, payload, comp_type) if self.t != 0 else 0
        ck = (ck + self.o.ContextModifier(self.base, off)) & 0xFFFFFFFF
        self.buf += payload + bytes([comp_type]) + struct.pack("<I", ck)
        self.layout.blocks.append((off, len(payload), kind))
        return off, len(payload)

    def footer(self, metaindex: Tuple[int, int], index: Tuple[int, int]) -> bytes:
        foff = len(self.buf)
        self.layout.footer_offset = foff
        if self.fv == 0:
            part2 = handle(*metaindex) + handle(*index)
            f = part2 + bytes(40 - len(part2)) + struct.pack("<Q", LEGACY_MAGIC)
        elif self.fv < 6:
            part2 = handle(*metaindex) + handle(*index)
            f = bytes([self.t]) + part2 + bytes(40 - len(part2)) + struct.pack("<IQ", self.fv, MAGIC)
        else:
            part2 = bytes([0x3E, 0x00, 0x7A, 0x00]) + struct.pack("<III", 0, self.base, metaindex[1]) + bytes(24)
            f = bytearray(bytes([self.t]) + part2 + struct.pack("<IQ", self.fv, MAGIC))
            ck = self.o.Builtin(self.t, bytes(f)) if self.t != 0 else 0
            ck = (ck + self.o.ContextModifier(self.base, foff)) & 0xFFFFFFFF
            f[5:9] = struct.pack("<I", ck)
            f = bytes(f)
        self.buf += f
        return f


def index_block(handles: List[Tuple[int, int]], keys: List[bytes], delta: bool,
                restart_interval: int, first_keys: Optional[List[bytes]] = None) -> bytes:
    """Index block (ShortenedIndexBuilder): key -> IndexValue."""
    entries, deltas = [], []
    prev = None
    for i, (h, k) in enumerate(zip(handles, keys)):
        v = handle(*h)
        dv = varsigned(h[1] - prev[1]) if prev is not None else None
        if first_keys is not None:
            fk = varint(len(first_keys[i])) + first_keys[i]
            v += fk
            if dv is not None:
                dv += fk
        entries.append((k, v))
        deltas.append(dv)
        prev = h
    return build_block(entries, restart_interval, deltas if delta else None)


def zlib_block(contents: bytes) -> bytes:
    """A block as the reference's Zlib_Compress stores it for
    format_version >= 2 (util/compression.h: compress_format_version 2 =
    varint32 uncompressed length, then a raw deflate stream; window_bits
    -14 by default, CompressionOptions)."""
    import zlib
    c = zlib.compressobj(6, zlib.DEFLATED, -14)
    return varint(len(contents)) + c.compress(contents) + c.flush()


def zlib_unblock(raw: bytes) -> bytes:
    """The inverse (UncompressBlockData's kZlibCompression case)."""
    import zlib
    n, k, shift = 0, 0, 0
    while True:
        b = raw[k]
        n |= (b & 127) << shift
        k += 1
        shift += 7
        if not b & 128:
            break
    out = zlib.decompress(raw[k:], -15)
    assert len(out) == n
    return out


def write_sst(oracle, *, seed: int = 1, n_data: int = 40, checksum_type: int = 1,
              format_version: int = 5, index_type: int = 0, delta: Optional[bool] = None,
              base_context_checksum: int = 0x5EED1234, partition_size: int = 8,
              meta: Tuple[str, ...] = ("filter", "range_del"), data_sizes=(1000, 9000),
              index_comp: int = 0) -> Tuple[bytes, Layout]:
    """An SST image: n_data data blocks of random payload sizes (index keys
    with shared prefixes), the meta blocks named in ``meta`` ("filter",
    "partitioned_filter", "range_del", "compression_dict"), the index
    (index_type 0 binary search, 1 hash, 2 two-level partitioned, 3 binary
    search with first key), properties, metaindex and footer.  index_comp:
    the compression type in the index blocks' trailers -- 2 (kZlibCompression)
    stores them really compressed (zlib_block), any other nonzero type keeps
    the bytes as they are (opaque to a reader without that codec)."""
    rnd = random.Random(seed)
    if delta is None:
        delta = format_version >= 4
    w = SstWriter(oracle, checksum_type, format_version, base_context_checksum)
    handles, keys, first_keys = [], [], []
    for i in range(n_data):
        n = rnd.randrange(*data_sizes)
        payload = bytes(rnd.getrandbits(8) for _ in range(n))
        handles.append(w.write_block(payload, "data"))
        keys.append(b"user_key_%08d" % (i * 7 + 3))
        first_keys.append(b"user_key_%08d" % (i * 7))
    metas: Dict[bytes, Tuple[int, int]] = {}
    if "filter" in meta:
        metas[b"fullfilter.rocksdb.BuiltinBloomFilter"] = w.write_block(
            bytes(rnd.getrandbits(8) for _ in range(700)), "filter")
    if "partitioned_filter" in meta:
        fh = [w.write_block(bytes(rnd.getrandbits(8) for _ in range(300 + 17 * j)), "filter_partition")
              for j in range(5)]
        fidx = index_block(fh, [b"fp%04d" % j for j in range(5)], delta, 2)
        metas[b"partitionedfilter.rocksdb.BuiltinBloomFilter"] = w.write_block(fidx, "filter_partition_index")
    # index (Finish: WriteIndexBlock after the filter)
    fk = first_keys if index_type == 3 else None

    def comp(b: bytes) -> bytes:
        return zlib_block(b) if index_comp == 2 else b
    if index_type == 2:
        parts = []
        for p in range(0, n_data, partition_size):
            blk = index_block(handles[p:p + partition_size], keys[p:p + partition_size], delta, 4)
            parts.append((w.write_block(comp(blk), "index_partition", index_comp),
                          keys[min(p + partition_size, n_data) - 1]))
        top = index_block([h for h, _ in parts], [k for _, k in parts], delta, 2)
        index_h = w.write_block(comp(top), "index", index_comp)
    else:
        # index_comp != 0: the index block's trailer names a compression
        # type (enable_index_compression); its bytes stay opaque here (no
        # compressor in this image) -- the checksum covers them as stored
        index_h = w.write_block(comp(index_block(handles, keys, delta, 4, fk)), "index", index_comp)
    if "compression_dict" in meta:
        metas[b"rocksdb.compression_dict"] = w.write_block(bytes(rnd.getrandbits(8) for _ in range(200)),
                                                            "compression_dict")
    if "range_del" in meta:
        metas[b"rocksdb.range_del"] = w.write_block(build_block([(b"a\x01" + bytes(7), b"z")]), "range_del")
    props = {
        b"rocksdb.block.based.table.index.type": struct.pack("<I", index_type),
        b"rocksdb.data.size": varint(sum(h[1] + TRAILER for h in handles)),
        b"rocksdb.index.key.is.user.key": varint(1),
        b"rocksdb.index.value.is.delta.encoded": varint(1 if delta else 0),
        b"rocksdb.num.data.blocks": varint(n_data),
    }
    metas[b"rocksdb.properties"] = w.write_block(build_block(sorted(props.items()), 1), "properties")
    if format_version >= 6:
        metas[b"rocksdb.index"] = index_h
    mi = build_block(sorted((k, handle(*v)) for k, v in metas.items()), 1)
    metaindex_h = w.write_block(mi, "metaindex")
    w.footer(metaindex_h, index_h if format_version < 6 else (0, 0))
    return bytes(w.buf), w.layout


def expected_blocks(layout: Layout) -> List[Tuple[int, int, str]]:
    """The parser's order: metaindex, meta blocks (metaindex order), index
    (+ partitions), data, filter partitions -- compared as sets per kind."""
    return sorted(layout.blocks)

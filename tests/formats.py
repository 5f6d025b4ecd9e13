"""Test-side builders for the reference's on-disk byte layouts, with every
checksum computed by the CPU oracle (test infrastructure only).

* ``wal_write``   -- db/log_writer.cc:79-175 AddRecord (fragmentation into
  32 KiB blocks, zero-padded block trailers) + 263-311 EmitPhysicalRecord.
* ``sst_blocks``  -- a run of block-based-table blocks, each
  [payload][compression type][LE32 checksum + context modifier]
  (table/block_based/block_based_table_builder.cc:1304-1358).
* ``folly_buffer`` -- the deterministic 4 MiB buffer of util/crc32c_test.cc:195-210.
"""
import struct

import numpy as np

K_BLOCK = 32768
K_HEADER = 7
K_RECYCLABLE_HEADER = 11

kFullType, kFirstType, kMiddleType, kLastType = 1, 2, 3, 4
kRecyclableFullType, kRecyclableFirstType, kRecyclableMiddleType, kRecyclableLastType = 5, 6, 7, 8


def splitmix_bytes(seed: int, nbytes: int) -> bytes:
    n8 = (nbytes + 7) // 8
    i = np.arange(1, n8 + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + i * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z.astype("<u8").tobytes()[:nbytes]


def folly_buffer(nbytes: int = 4 * 1024 * 1024) -> bytes:
    """util/crc32c_test.cc:181-210: word[0] = 0, word[i+1] = fnv64(bytes of
    word[i]) with FNV_64_HASH_START and *signed* chars."""
    start = 14695981039346656037
    m = (1 << 64) - 1
    words = [0]
    prev = b"\0" * 8
    for _ in range(nbytes // 8 - 1):
        h = start
        for ch in prev:
            h = (h + (h << 1) + (h << 4) + (h << 5) + (h << 7) + (h << 8) + (h << 40)) & m
            h ^= (ch - 256 if ch >= 128 else ch) & m
        words.append(h)
        prev = struct.pack("<Q", h)
    return struct.pack(f"<{len(words)}Q", *words)


class WalWriter:
    """db/log_writer.cc Writer, in memory (like log_test.cc's StringSink)."""

    def __init__(self, oracle, log_number=0, recycle=False):
        self.o = oracle
        self.log_number = log_number & 0xFFFFFFFF
        self.recycle = recycle
        self.buf = bytearray()
        self.block_offset = 0
        self.records = []  # (file offset of header, type, payload len)

    def add_record(self, payload: bytes):
        hs = K_RECYCLABLE_HEADER if self.recycle else K_HEADER
        left = len(payload)
        ptr = 0
        begin = True
        while True:
            leftover = K_BLOCK - self.block_offset
            if leftover < hs:
                self.buf += b"\0" * leftover
                self.block_offset = 0
            avail = K_BLOCK - self.block_offset - hs
            frag = min(left, avail)
            end = left == frag
            if begin and end:
                t = kRecyclableFullType if self.recycle else kFullType
            elif begin:
                t = kRecyclableFirstType if self.recycle else kFirstType
            elif end:
                t = kRecyclableLastType if self.recycle else kLastType
            else:
                t = kRecyclableMiddleType if self.recycle else kMiddleType
            self.emit(t, payload[ptr:ptr + frag])
            ptr += frag
            left -= frag
            begin = False
            if left <= 0:
                break

    def emit(self, t: int, frag: bytes):
        n = len(frag)
        recyclable = t >= kRecyclableFullType and t <= kRecyclableLastType
        crc = self.o.WalRecordCrc(t, frag, recyclable, self.log_number)
        hdr = struct.pack("<IHB", crc, n, t)
        if recyclable:
            hdr += struct.pack("<I", self.log_number)
        self.records.append((len(self.buf), t, n))
        self.buf += hdr + frag
        self.block_offset += len(hdr) + n


def wal_expected_blocks(data: bytes, log_number: int, oracle):
    """Walk a WAL image block by block as db/log_reader.cc:450-584 does with
    checksums on; returns [(records_ok, status, stop_offset, bytes_ok)]."""
    out = []
    nb = (len(data) + K_BLOCK - 1) // K_BLOCK
    for b in range(nb):
        blk = data[b * K_BLOCK:(b + 1) * K_BLOCK]
        last = (b + 1) * K_BLOCK >= len(data)
        pos = ok = bytes_ok = 0
        status = 0
        while True:
            left = len(blk) - pos
            if left < K_HEADER:
                if last and left > 0:
                    status = 5
                break
            h = blk[pos:]
            length = h[4] | (h[5] << 8)
            t = h[6]
            hs = K_HEADER
            if 5 <= t <= 8 or t == 11:
                hs = K_RECYCLABLE_HEADER
                if left < hs:
                    if last:
                        status = 5
                    break
                if struct.unpack_from("<I", h, 7)[0] != (log_number & 0xFFFFFFFF):
                    status = 4
                    break
            if hs + length > left:
                status = 2
                break
            if t == 0 and length == 0:
                status = 3
                break
            stored = struct.unpack_from("<I", h, 0)[0]
            actual = oracle.Value(bytes(h[6:hs + length]))
            if oracle.Unmask(stored) != actual:
                status = 1
                break
            ok += 1
            pos += hs + length
            bytes_ok += hs + length
        out.append((ok, status, pos if status else len(blk), bytes_ok))
    return out


def sst_blocks(oracle, payloads, checksum_type, comp_types, base_context_checksum=0,
               file_start=0):
    """Lay the payloads out back to back as a block-based table does; returns
    (image bytes, payload offsets, payload lengths)."""
    img = bytearray()
    offs, lens = [], []
    for p, ct in zip(payloads, comp_types):
        off = file_start + len(img)
        ck = oracle.BuiltinLast(checksum_type, p, ct)
        ck = (ck + oracle.ContextModifier(base_context_checksum, off)) & 0xFFFFFFFF
        offs.append(len(img))
        lens.append(len(p))
        img += p + bytes([ct]) + struct.pack("<I", ck)
    return bytes(img), offs, lens

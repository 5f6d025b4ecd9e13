"""Whole-SST-file checksum verification: the host reads
the block-based table's footer, metaindex, properties and index blocks
(mck_sst_list_blocks, C++ in the engine) and every listed block is then
verified on the GPU in ONE batched call (mck_sst_verify_batch), plus the
format_version 6 footer checksum (mck_sst_verify_footer).

Mirrors BlockBasedTable::VerifyChecksum (table/block_based/
block_based_table_reader.cc:2336-2500): the result is the reference's
Status -- OK, or Corruption with VerifyBlockChecksum's message for the first
bad block (reader_common.cc:45-58) or Footer::DecodeFrom's message.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import List, Optional, Tuple

import numpy as np

from ._lib import check, lib
from .checksum import ChecksumType, Spans, Status, crc32c, sst_verify_batch

BLOCK_KINDS = {0: "data", 1: "index", 2: "index_partition", 3: "metaindex", 4: "properties",
               5: "filter", 6: "filter_partition_index", 7: "filter_partition", 8: "range_del",
               9: "compression_dict", 10: "other_meta"}

MCK_ECORRUPT, MCK_ENOTSUP = -5, -6


class mck_sst_footer(ctypes.Structure):
    _fields_ = [("magic", ctypes.c_uint64), ("format_version", ctypes.c_uint32),
                ("checksum_type", ctypes.c_int32), ("base_context_checksum", ctypes.c_uint32),
                ("footer_checksum", ctypes.c_uint32), ("block_trailer_size", ctypes.c_uint32),
                ("has_index_handle", ctypes.c_uint32), ("footer_offset", ctypes.c_uint64),
                ("metaindex_offset", ctypes.c_uint64), ("metaindex_size", ctypes.c_uint64),
                ("index_offset", ctypes.c_uint64), ("index_size", ctypes.c_uint64),
                ("index_type", ctypes.c_uint32), ("index_value_is_delta_encoded", ctypes.c_uint32)]


class mck_sst_block(ctypes.Structure):
    _fields_ = [("offset", ctypes.c_uint64), ("size", ctypes.c_uint64), ("kind", ctypes.c_int32),
                ("reserved", ctypes.c_uint32)]


@dataclass
class SstBlock:
    offset: int
    size: int
    kind: str


class SstError(RuntimeError):
    def __init__(self, rc: int, msg: str):
        super().__init__(msg)
        self.rc = rc
        self.status = Status("Corruption" if rc == MCK_ECORRUPT else
                             "Not implemented" if rc == MCK_ENOTSUP else "Invalid argument", msg)


def _err() -> str:
    return lib.mck_last_error().decode(errors="replace")


def decode_footer(image: bytes) -> mck_sst_footer:
    """table/format.cc Footer::DecodeFrom on the file's last 53 bytes."""
    tail = bytes(image[-53:]) if len(image) >= 53 else bytes(image)
    f = mck_sst_footer()
    rc = lib.mck_sst_decode_footer(tail, len(tail), len(image) - len(tail), ctypes.addressof(f))
    if rc:
        raise SstError(rc, _err())
    return f


# int (*)(void* ctx, uint8_t type, uint64_t offset, const void* raw, uint64_t
#        raw_size, const void** out, uint64_t* out_size)  (mck_sst_uncompress_fn)
UNCOMPRESS_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_uint8, ctypes.c_uint64, ctypes.c_void_p,
                                 ctypes.c_uint64, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_uint64))


def list_blocks(image: bytes, uncompress=None) -> Tuple[mck_sst_footer, List[SstBlock]]:
    """Every checksummed block of the SST image (host bytes), in
    VerifyChecksum order: metaindex, meta blocks, index (+ partitions), data,
    filter partitions.  ``uncompress(type, offset, raw: bytes) -> bytes``
    supplies the contents of compressed index / meta blocks
    (mck_sst_list_blocks_uncompress; the reference's UncompressBlockData in a
    real integration); without it such a table raises MCK_ENOTSUP.  An
    exception in the callback fails the listing (MCK_ECORRUPT)."""
    buf = bytes(image)
    held = []  # the uncompressed blocks, alive until the call returns

    def cb(_ctx, ctype, off, raw, raw_size, out, out_size):
        try:
            data = bytes(uncompress(int(ctype), int(off), ctypes.string_at(raw, raw_size)))
        except Exception:  # the listing reports it; never unwind through C
            return MCK_ECORRUPT
        b = ctypes.create_string_buffer(data, max(len(data), 1))
        held.append(b)
        out[0] = ctypes.cast(b, ctypes.c_void_p)
        out_size[0] = len(data)
        return 0

    fn = UNCOMPRESS_FN(cb) if uncompress is not None else None  # (kept alive for the calls)
    fnp = ctypes.cast(fn, ctypes.c_void_p) if fn is not None else None

    def call(arr, cap, f, n):
        held.clear()
        return lib.mck_sst_list_blocks_uncompress(buf, len(buf), fnp, None, ctypes.addressof(f), arr, cap,
                                                  ctypes.addressof(n))

    f = mck_sst_footer()
    n = ctypes.c_uint64()
    rc = call(None, 0, f, n)
    if rc:
        raise SstError(rc, _err())
    arr = (mck_sst_block * max(n.value, 1))()
    rc = call(ctypes.addressof(arr), n.value, f, n)
    if rc:
        raise SstError(rc, _err())
    return f, [SstBlock(int(b.offset), int(b.size), BLOCK_KINDS.get(b.kind, str(b.kind)))
               for b in arr[:n.value]]


def index_handles(contents: bytes, value_delta_encoded: bool, index_type: int = 0,
                  kind: str = "data") -> List[SstBlock]:
    """The handles one uncompressed index block lists (mck_sst_index_handles),
    for a reader that already holds its contents."""
    kinds = {v: k for k, v in BLOCK_KINDS.items()}
    buf = bytes(contents)
    n = ctypes.c_uint64()
    rc = lib.mck_sst_index_handles(buf, len(buf), int(bool(value_delta_encoded)), index_type, kinds[kind], None, 0,
                                   ctypes.addressof(n))
    if rc:
        raise SstError(rc, _err())
    arr = (mck_sst_block * max(n.value, 1))()
    rc = lib.mck_sst_index_handles(buf, len(buf), int(bool(value_delta_encoded)), index_type, kinds[kind],
                                   ctypes.addressof(arr), n.value, ctypes.addressof(n))
    if rc:
        raise SstError(rc, _err())
    return [SstBlock(int(b.offset), int(b.size), BLOCK_KINDS.get(b.kind, str(b.kind))) for b in arr[:n.value]]


def VerifyChecksum(image: bytes, file_name: str = "", stream=None, device=None,
                   per_block: Optional[list] = None, uncompress=None) -> Status:
    """BlockBasedTable::VerifyChecksum of a whole SST image: parse on the
    host, one batched GPU verify of every block.  ``per_block`` (a list)
    receives (SstBlock, Status) for every block; ``uncompress`` as in
    list_blocks (compressed index / meta blocks)."""
    import torch
    try:
        f, blocks = list_blocks(image, uncompress)
    except SstError as e:
        return e.status
    tail = bytes(image[f.footer_offset:f.footer_offset + 53])
    rc = lib.mck_sst_verify_footer(tail, ctypes.addressof(f))
    if rc == MCK_ECORRUPT:
        return Status.Corruption(_err())
    check(rc, "mck_sst_verify_footer")
    return VerifyBlocks(image, blocks, f.checksum_type, f.base_context_checksum, file_name, stream, device,
                        per_block)


def VerifyBlocks(image, blocks, checksum_type: int, base_context_checksum: int = 0, file_name: str = "",
                 stream=None, device=None, per_block: Optional[list] = None) -> Status:
    """The lower-level form of VerifyChecksum: the caller names the blocks
    (``blocks``: (offset, size[, kind]) handles, as its own IndexBlockIter /
    metaindex walk found them) and every one is verified in one GPU batch,
    compressed or not -- the checksum covers the stored (compressed) bytes
    and the type byte.  This is the path for tables whose index or meta
    blocks are compressed (enable_index_compression defaults to true,
    include/rocksdb/table.h:541), which list_blocks cannot parse."""
    import torch
    blocks = [b if isinstance(b, SstBlock) else SstBlock(int(b[0]), int(b[1]), b[2] if len(b) > 2 else "block")
              for b in blocks]
    if not blocks:
        return Status.OK()
    dev = torch.device("cuda") if device is None else device
    img = torch.frombuffer(bytearray(bytes(image) + bytes(64)), dtype=torch.uint8).to(dev)
    offs = torch.tensor([b.offset for b in blocks], dtype=torch.int64, device=dev)
    lens = torch.tensor([b.size for b in blocks], dtype=torch.int32, device=dev)
    sp = Spans(img, len(blocks), offsets=offs, lengths=lens)
    ct = ChecksumType(checksum_type)
    mm, comp, stored, _ = sst_verify_batch(ct, sp, base_context_checksum=base_context_checksum,
                                           stream=stream)
    mm = mm.cpu().numpy()
    comp = comp.cpu().numpy().view(np.uint32)
    stored = stored.cpu().numpy().view(np.uint32)
    first = Status.OK()
    for i, b in enumerate(blocks):
        st = Status.OK()
        if mm[i]:
            s_v, c_v = int(stored[i]), int(comp[i])
            if ct == ChecksumType.kCRC32c:  # reader_common.cc:51-55: unmask for people
                s_v, c_v = crc32c.Unmask(s_v), crc32c.Unmask(c_v)
            ctx = "(context removed)" if base_context_checksum else ""
            st = Status.Corruption(f"block checksum mismatch: stored{ctx} = {s_v}, computed = {c_v}, "
                                   f"type = {int(ct)}  in {file_name} offset {b.offset} size {b.size}")
            if first.ok():
                first = st
        if per_block is not None:
            per_block.append((b, st))
    return first


__all__ = ["list_blocks", "index_handles", "decode_footer", "VerifyChecksum", "VerifyBlocks", "SstBlock", "SstError", "BLOCK_KINDS"]

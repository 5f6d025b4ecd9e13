"""Host-side mirror of the reference's block-checksum interface, over the
engine's C ABI.

Names, argument meaning and error behaviour follow the reference:

* ``crc32c.Value / Extend / Mask / Unmask / Crc32cCombine``  -- util/crc32c.h:21-53
* ``XXH3_64bits``                                            -- util/xxhash.h:5329
* ``ChecksumType``                                           -- include/rocksdb/table.h:69-75
* ``ComputeBuiltinChecksum[WithLastByte]``                   -- table/format.cc:578-645
* ``ChecksumModifierForContext``                             -- table/format.h:119-146
* ``VerifyBlockChecksum`` (returns a ``Status``)             -- table/block_based/reader_common.cc:26-63

Scalar functions take host ``bytes`` and hash them on the GPU (synchronous);
the ``*_batch`` functions take device-resident torch tensors and run
asynchronously on the current HIP stream.  The u32 algebra (Mask, Unmask,
Combine, context modifier) runs on the host, as in the reference.
"""
from __future__ import annotations

import ctypes
import enum
from dataclasses import dataclass
from typing import NamedTuple, Optional

from ._lib import check, lib, mck_spans, mck_wal_block_result

MCK_EAGAIN = -7  # mck.h: call again after supplying what the call asked for

# ---------------------------------------------------------------------------
# enums / status
# ---------------------------------------------------------------------------


class ChecksumType(enum.IntEnum):
    """include/rocksdb/table.h:69-75"""
    kNoChecksum = 0
    kCRC32c = 1
    kxxHash = 2
    kxxHash64 = 3
    kXXH3 = 4


class WalStatus(enum.IntEnum):
    """Why a WAL block walk stopped (db/log_reader.h ReadPhysicalRecord codes)."""
    kOk = 0
    kBadRecordChecksum = 1
    kBadRecordLen = 2
    kBadRecord = 3        # kZeroType with length 0
    kOldRecord = 4
    kBadHeader = 5


@dataclass(frozen=True)
class Status:
    """The slice of rocksdb::Status the checksum path produces."""
    code: str = "OK"
    message: str = ""

    def ok(self) -> bool:
        return self.code == "OK"

    def IsCorruption(self) -> bool:
        return self.code == "Corruption"

    def ToString(self) -> str:
        return "OK" if self.ok() else f"{self.code}: {self.message}"

    @staticmethod
    def OK() -> "Status":
        return Status()

    @staticmethod
    def Corruption(msg: str) -> "Status":
        return Status("Corruption", msg)


@dataclass(frozen=True)
class Footer:
    """The two footer fields VerifyBlockChecksum reads (table/format.h)."""
    checksum_type: ChecksumType = ChecksumType.kXXH3
    base_context_checksum: int = 0


def _buf(data):
    if isinstance(data, str):
        data = data.encode()
    b = bytes(data)
    return b, len(b)


def _err():
    return lib.mck_last_error().decode(errors="replace")


def _checked(v):
    e = _err()
    if e:
        raise RuntimeError(f"speedb_amd: {e}")
    return v


def _scalar(fn, ctype, *args):
    """A scalar call through its *_r variant (the plain shims abort on a
    device error by default, mck_set_shim_error_policy): the result, or
    RuntimeError with mck_last_error()."""
    out = ctype(0)
    rc = fn(*args, ctypes.byref(out))
    if rc != 0:
        raise RuntimeError(f"speedb_amd: {_err()} ({rc})")
    return out.value


# ---------------------------------------------------------------------------
# scalar API (util/crc32c.h, util/xxhash.h, table/format.cc)
# ---------------------------------------------------------------------------


class crc32c:  # noqa: N801 -- mirrors the reference's namespace
    kMaskDelta = 0xA282EAD8

    @staticmethod
    def Extend(init_crc: int, data) -> int:
        b, n = _buf(data)
        return _scalar(lib.mck_crc32c_extend_r, ctypes.c_uint32, init_crc & 0xFFFFFFFF, b, n)

    @staticmethod
    def Value(data) -> int:
        b, n = _buf(data)
        return _scalar(lib.mck_crc32c_value_r, ctypes.c_uint32, b, n)

    @staticmethod
    def Mask(crc: int) -> int:
        return lib.mck_crc32c_mask(crc & 0xFFFFFFFF)

    @staticmethod
    def Unmask(masked_crc: int) -> int:
        return lib.mck_crc32c_unmask(masked_crc & 0xFFFFFFFF)

    @staticmethod
    def Crc32cCombine(crc1: int, crc2: int, crc2len: int) -> int:
        return lib.mck_crc32c_combine(crc1 & 0xFFFFFFFF, crc2 & 0xFFFFFFFF, crc2len)


def XXH3_64bits(data) -> int:
    b, n = _buf(data)
    return _scalar(lib.mck_xxh3_64_r, ctypes.c_uint64, b, n)


def ComputeBuiltinChecksum(checksum_type: int, data) -> int:
    b, n = _buf(data)
    return _scalar(lib.mck_builtin_checksum_r, ctypes.c_uint32, int(checksum_type), b, n)


def ComputeBuiltinChecksumWithLastByte(checksum_type: int, data, last_byte) -> int:
    b, n = _buf(data)
    if isinstance(last_byte, int):
        last_byte = bytes([last_byte & 0xFF])
    return _scalar(lib.mck_builtin_checksum_with_last_byte_r, ctypes.c_uint32, int(checksum_type), b, n, last_byte)


def NPHash64(data, seed: int = 0) -> int:
    """util/hash.h:45 NPHash64 == util/hash.cc:81 Hash64: XXPH3 (the XXH3
    preview), seeded -- computed on the GPU."""
    b, n = _buf(data)
    return _scalar(lib.mck_np_hash64_r, ctypes.c_uint64, b, n, seed & 0xFFFFFFFFFFFFFFFF)


Hash64 = NPHash64


def ChecksumModifierForContext(base_context_checksum: int, offset: int) -> int:
    return lib.mck_context_modifier(base_context_checksum & 0xFFFFFFFF, offset)


def _decode_fixed32(b: bytes, pos: int) -> int:
    return int.from_bytes(b[pos:pos + 4], "little")


def VerifyBlockChecksum(footer: Footer, data, block_size: int, file_name: str,
                        offset: int) -> Status:
    """table/block_based/reader_common.cc:26-63.  ``data`` holds the block
    payload followed by its 5-byte trailer."""
    b, _ = _buf(data)
    ctype = ChecksumType(footer.checksum_type)
    length = block_size + 1
    stored = _decode_fixed32(b, length)
    computed = ComputeBuiltinChecksum(ctype, b[:length])
    modifier = ChecksumModifierForContext(footer.base_context_checksum, offset)
    stored = (stored - modifier) & 0xFFFFFFFF
    if stored == computed:
        return Status.OK()
    if ctype == ChecksumType.kCRC32c:
        stored = crc32c.Unmask(stored)
        computed = crc32c.Unmask(computed)
    return Status.Corruption(
        "block checksum mismatch: stored" + ("(context removed)" if modifier else "") +
        f" = {stored}, computed = {computed}, type = {int(ctype)}  in {file_name} "
        f"offset {offset} size {block_size}")


# ---------------------------------------------------------------------------
# batched device API (torch tensors on the GPU)
# ---------------------------------------------------------------------------

def _torch():
    import torch
    return torch


def _ptr(t) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _stream(stream) -> Optional[int]:
    torch = _torch()
    if stream is None:
        stream = torch.cuda.current_stream()
    return stream.cuda_stream


@dataclass
class Spans:
    """mck_spans over a device byte tensor.  span i = base[off_i : off_i+len_i]
    with off_i = offsets[i] (int64 tensor) or i*stride and len_i = lengths[i]
    (int32 tensor) or ``length``."""
    base: object
    count: int
    offsets: object = None
    lengths: object = None
    stride: int = 0
    length: int = 0

    def c(self) -> mck_spans:
        for t in (self.offsets, self.lengths):
            if t is not None and not t.is_contiguous():
                raise ValueError("offsets/lengths must be contiguous")
        return mck_spans(self.base.data_ptr(), _ptr(self.offsets), _ptr(self.lengths),
                         self.stride, self.length, self.count)

    @staticmethod
    def uniform(base, block: int, count: Optional[int] = None) -> "Spans":
        if count is None:
            count = base.numel() // block
        return Spans(base, count, stride=block, length=block)


def _empty(count, dtype, device):
    return _torch().empty(count, dtype=dtype, device=device)


def crc32c_batch(spans: Spans, init_crcs=None, mask: bool = False, out=None, stream=None):
    """out[i] = crc32c::Extend(init_crcs[i] or 0, span i) (Mask()ed if mask).
    Returns an int32 tensor holding the u32 bit patterns."""
    torch = _torch()
    if out is None:
        out = _empty(spans.count, torch.int32, spans.base.device)
    s = spans.c()
    check(lib.mck_crc32c_batch(ctypes.byref(s), _ptr(init_crcs), 1 if mask else 0,
                               out.data_ptr(), _stream(stream)), "mck_crc32c_batch")
    return out


def xxh3_64_batch(spans: Spans, out=None, stream=None):
    torch = _torch()
    if out is None:
        out = _empty(spans.count, torch.int64, spans.base.device)
    s = spans.c()
    check(lib.mck_xxh3_64_batch(ctypes.byref(s), out.data_ptr(), _stream(stream)),
          "mck_xxh3_64_batch")
    return out


def xxh32_batch(spans: Spans, seed: int = 0, out=None, stream=None):
    torch = _torch()
    if out is None:
        out = _empty(spans.count, torch.int32, spans.base.device)
    s = spans.c()
    check(lib.mck_xxh32_batch(ctypes.byref(s), seed, out.data_ptr(), _stream(stream)),
          "mck_xxh32_batch")
    return out


def xxh64_batch(spans: Spans, seed: int = 0, out=None, stream=None):
    torch = _torch()
    if out is None:
        out = _empty(spans.count, torch.int64, spans.base.device)
    s = spans.c()
    check(lib.mck_xxh64_batch(ctypes.byref(s), seed, out.data_ptr(), _stream(stream)),
          "mck_xxh64_batch")
    return out


def builtin_checksum_batch(checksum_type: int, spans: Spans, last_bytes=None, out=None,
                           stream=None):
    torch = _torch()
    if out is None:
        out = _empty(spans.count, torch.int32, spans.base.device)
    s = spans.c()
    check(lib.mck_builtin_checksum_batch(int(checksum_type), ctypes.byref(s), _ptr(last_bytes),
                                         out.data_ptr(), _stream(stream)),
          "mck_builtin_checksum_batch")
    return out


def sst_trailer_batch(checksum_type: int, payloads: Spans, comp_types, file_offsets=None,
                      base_context_checksum: int = 0, out=None, stream=None):
    torch = _torch()
    if out is None:
        out = _empty(payloads.count, torch.int32, payloads.base.device)
    s = payloads.c()
    check(lib.mck_sst_trailer_batch(int(checksum_type), ctypes.byref(s), _ptr(comp_types),
                                    _ptr(file_offsets), base_context_checksum & 0xFFFFFFFF,
                                    out.data_ptr(), _stream(stream)), "mck_sst_trailer_batch")
    return out


def sst_verify_batch(checksum_type: int, payloads: Spans, file_offsets=None,
                     base_context_checksum: int = 0, stream=None, outs=None, with_count=True):
    """Returns (mismatch uint8, computed int32, stored int32, mismatch_count
    int32[1] or None).  ``outs`` = preallocated (mismatch, computed, stored)."""
    torch = _torch()
    dev = payloads.base.device
    if outs is None:
        outs = (_empty(payloads.count, torch.uint8, dev), _empty(payloads.count, torch.int32, dev),
                _empty(payloads.count, torch.int32, dev))
    mismatch, computed, stored = outs
    count = torch.zeros(1, dtype=torch.int32, device=dev) if with_count else None
    s = payloads.c()
    check(lib.mck_sst_verify_batch(int(checksum_type), ctypes.byref(s), _ptr(file_offsets),
                                   base_context_checksum & 0xFFFFFFFF, mismatch.data_ptr(),
                                   _ptr(computed), _ptr(stored), _ptr(count),
                                   _stream(stream)), "mck_sst_verify_batch")
    return mismatch, computed, stored, count


def wal_record_crc_batch(payloads: Spans, types, log_number: int = 0, out=None, stream=None):
    torch = _torch()
    if out is None:
        out = _empty(payloads.count, torch.int32, payloads.base.device)
    s = payloads.c()
    check(lib.mck_wal_record_crc_batch(ctypes.byref(s), types.data_ptr(), log_number & 0xFFFFFFFF,
                                       out.data_ptr(), _stream(stream)),
          "mck_wal_record_crc_batch")
    return out


def wal_verify_batch(wal, nbytes: Optional[int] = None, log_number: int = 0, stream=None,
                     out=None):
    """Returns an int32 tensor [nblocks, 4]: records_ok, status, stop_offset, bytes_ok."""
    torch = _torch()
    if nbytes is None:
        nbytes = wal.numel()
    nblocks = (nbytes + 32767) // 32768
    res = out if out is not None else torch.empty((nblocks, 4), dtype=torch.int32, device=wal.device)
    check(lib.mck_wal_verify_batch(wal.data_ptr(), nbytes, log_number & 0xFFFFFFFF,
                                   res.data_ptr(), _stream(stream)), "mck_wal_verify_batch")
    return res


def wal_plan_records(wal: bytes, log_number: int = 0):
    """mck_wal_plan_records: every physical record of a host WAL image as a
    numpy uint32 [count, 4] array of mck_wal_rec_desc (payload offset low,
    offset high | type << 16 | MCK_WAL_REC_HASH, length, stored CRC)."""
    import numpy as np
    buf = bytes(wal)
    n = ctypes.c_uint64()
    check(lib.mck_wal_plan_records(buf, len(buf), log_number & 0xFFFFFFFF, None, 0, ctypes.byref(n)),
          "mck_wal_plan_records")
    out = np.zeros((max(n.value, 1), 4), dtype=np.uint32)
    check(lib.mck_wal_plan_records(buf, len(buf), log_number & 0xFFFFFFFF, out.ctypes.data, n.value,
                                   ctypes.byref(n)), "mck_wal_plan_records")
    return out[:n.value]


def wal_recover_batch(wal, recs, log_number: int = 0, ok=None, hashes=None, stream=None):
    """mck_wal_recover_batch: for every record of a plan (``recs``: a device
    int32/uint32 tensor [count, 4] of mck_wal_rec_desc, e.g. from
    wal_plan_records), its CRC verdict (uint8 [count], 1 = holds) and, for
    the records flagged MCK_WAL_REC_HASH, the XXH3_64bits of its payload
    (int64 [count]) -- one read of the image.  Returns (ok, hashes)."""
    torch = _torch()
    n = int(recs.shape[0])
    ok = ok if ok is not None else torch.zeros(max(n, 1), dtype=torch.uint8, device=wal.device)
    hashes = hashes if hashes is not None else torch.zeros(max(n, 1), dtype=torch.int64, device=wal.device)
    check(lib.mck_wal_recover_batch(wal.data_ptr(), recs.data_ptr(), n, log_number & 0xFFFFFFFF, ok.data_ptr(),
                                    hashes.data_ptr(), _stream(stream)), "mck_wal_recover_batch")
    return ok[:n], hashes[:n]


def np_hash64_batch(spans: Spans, seed: int = 0, out=None, stream=None):
    """out[i] = NPHash64(span i, seed) (int64 tensor of the u64 bit patterns)."""
    torch = _torch()
    if out is None:
        out = _empty(spans.count, torch.int64, spans.base.device)
    s = spans.c()
    check(lib.mck_np_hash64_batch(ctypes.byref(s), seed & 0xFFFFFFFFFFFFFFFF, out.data_ptr(),
                                  _stream(stream)), "mck_np_hash64_batch")
    return out


class ProtectionKind(enum.IntEnum):
    """Which db/kv_checksum.h ProtectionInfo64 value a batch computes."""
    KV = 0    # ProtectKV(key, value)
    KVO = 1   # ProtectKVO(key, value, op_type)
    KVOS = 2  # ProtectKVO(...).ProtectS(seqno)
    KVOC = 3  # ProtectKVO(...).ProtectC(column_family_id)


def kv_protect_batch(kind: int, keys: Spans, values: Spans, op_types=None, extras=None, out=None,
                     stream=None):
    """Per-KV protection values (u64 bit patterns in an int64 tensor)."""
    torch = _torch()
    if out is None:
        out = _empty(values.count, torch.int64, values.base.device)
    k, v = keys.c(), values.c()
    check(lib.mck_kv_protect_batch(int(kind), ctypes.byref(k), ctypes.byref(v), _ptr(op_types),
                                   _ptr(extras), out.data_ptr(), _stream(stream)),
          "mck_kv_protect_batch")
    return out


def kv_protect_verify_batch(kind: int, keys: Spans, values: Spans, stored, prot_bytes: int,
                            op_types=None, extras=None, stream=None):
    """ProtectionInfo::Verify for every KV against ``stored`` (uint8 tensor of
    count*prot_bytes).  Returns (mismatch uint8, mismatch_count int32[1],
    computed int64)."""
    torch = _torch()
    dev = values.base.device
    mismatch = _empty(values.count, torch.uint8, dev)
    computed = _empty(values.count, torch.int64, dev)
    count = torch.zeros(1, dtype=torch.int32, device=dev)
    k, v = keys.c(), values.c()
    check(lib.mck_kv_protect_verify_batch(int(kind), ctypes.byref(k), ctypes.byref(v), _ptr(op_types),
                                          _ptr(extras), stored.data_ptr(), prot_bytes,
                                          mismatch.data_ptr(), count.data_ptr(), computed.data_ptr(),
                                          _stream(stream)), "mck_kv_protect_verify_batch")
    return mismatch, count, computed


def crc32c_long(data, nbytes: Optional[int] = None, init_crc: int = 0, offset: int = 0,
                scratch=None, out=None, stream=None):
    """crc32c::Extend(init_crc, data[offset : offset+nbytes]) of ONE long
    device-resident span (a whole file image), computed as 64 KiB pieces in
    parallel + the Crc32cCombine algebra on the device (mck_crc32c_long).
    Returns a 1-element int32 tensor (u32 bit pattern), asynchronously."""
    torch = _torch()
    if nbytes is None:
        nbytes = data.numel() - offset
    words = int(lib.mck_crc32c_long_scratch_words(nbytes))
    if scratch is None:
        scratch = _empty(max(words, 1), torch.int32, data.device)
    if scratch.numel() < words:
        raise ValueError(f"scratch needs {words} int32 words")
    if out is None:
        out = _empty(1, torch.int32, data.device)
    check(lib.mck_crc32c_long(data.data_ptr() + offset, nbytes, init_crc & 0xFFFFFFFF,
                              scratch.data_ptr(), out.data_ptr(), _stream(stream)), "mck_crc32c_long")
    return out


# ---------------------------------------------------------------------------
# whole-file checksums: include/rocksdb/file_checksum.h:50-90,
# util/file_checksum_helper.h:22-60
# ---------------------------------------------------------------------------

kUnknownFileChecksum = ""
kUnknownFileChecksumFuncName = "Unknown"
kStandardDbFileChecksumFuncName = "FileChecksumCrc32c"


@dataclass
class FileChecksumGenContext:
    """include/rocksdb/file_checksum.h:31-38"""
    file_name: str = ""
    requested_checksum_func_name: str = ""


class FileChecksumGenCrc32c:
    """util/file_checksum_helper.h:22-52: checksum_ = crc32c::Extend over every
    Update (starting at 0); Finalize stores it as 4 big-endian bytes.

    Update() takes host bytes (one synchronous device call; inputs over 1 MiB
    go through the long-span path).  UpdateDevice() takes a device-resident
    tensor region and runs mck_crc32c_long on it -- the file-writer handoff
    when the file's bytes are already in HBM."""

    def __init__(self, context: Optional[FileChecksumGenContext] = None):
        self._checksum = 0
        self._str: Optional[bytes] = None

    def Update(self, data) -> None:
        assert self._str is None, "Update after Finalize"
        self._checksum = crc32c.Extend(self._checksum, data)

    def UpdateDevice(self, data, nbytes: Optional[int] = None, offset: int = 0, stream=None) -> None:
        assert self._str is None, "Update after Finalize"
        out = crc32c_long(data, nbytes, self._checksum, offset=offset, stream=stream)
        self._checksum = int(out.cpu().item()) & 0xFFFFFFFF

    def Finalize(self) -> None:
        assert self._str is None
        self._str = self._checksum.to_bytes(4, "big")  # PutFixed32(EndianSwapValue)

    def GetChecksum(self) -> bytes:
        assert self._str is not None
        return self._str

    def Name(self) -> str:
        return "FileChecksumCrc32c"


class FileChecksumGenCrc32cFactory:
    """util/file_checksum_helper.h:54-72"""

    def CreateFileChecksumGenerator(self, context: FileChecksumGenContext):
        if context.requested_checksum_func_name in ("", "FileChecksumCrc32c"):
            return FileChecksumGenCrc32c(context)
        return None

    @staticmethod
    def kClassName() -> str:
        return "FileChecksumGenCrc32cFactory"

    def Name(self) -> str:
        return self.kClassName()


def GetFileChecksumGenCrc32cFactory() -> FileChecksumGenCrc32cFactory:
    """util/file_checksum_helper.cc GetFileChecksumGenCrc32cFactory()"""
    return _DEFAULT_FACTORY


_DEFAULT_FACTORY = FileChecksumGenCrc32cFactory()


def device_count() -> int:
    return lib.mck_device_count()


__all__ = [
    "ChecksumType", "WalStatus", "Status", "Footer", "crc32c", "XXH3_64bits",
    "ComputeBuiltinChecksum", "ComputeBuiltinChecksumWithLastByte",
    "ChecksumModifierForContext", "VerifyBlockChecksum", "Spans", "crc32c_batch",
    "xxh3_64_batch", "xxh32_batch", "xxh64_batch", "builtin_checksum_batch",
    "sst_trailer_batch", "sst_verify_batch", "wal_record_crc_batch", "wal_verify_batch",
    "device_count", "mck_wal_block_result", "NPHash64", "Hash64", "np_hash64_batch",
    "ProtectionKind", "kv_protect_batch", "kv_protect_verify_batch", "crc32c_long",
    "FileChecksumGenContext", "FileChecksumGenCrc32c", "FileChecksumGenCrc32cFactory",
    "GetFileChecksumGenCrc32cFactory", "kStandardDbFileChecksumFuncName",
    "kUnknownFileChecksum", "kUnknownFileChecksumFuncName",
]


# ---------------------------------------------------------------------------
# device WAL writer (db/log_writer.cc:79-175 AddRecord + :263-311
# EmitPhysicalRecord, as one group-commit batch)
# ---------------------------------------------------------------------------

class mck_wal_fragment(ctypes.Structure):
    _fields_ = [("src_off", ctypes.c_uint64), ("dst_off", ctypes.c_uint64), ("length", ctypes.c_uint32),
                ("type", ctypes.c_uint8), ("pad", ctypes.c_uint8), ("reserved", ctypes.c_uint16)]


def wal_plan(src_offsets, lengths, block_offset: int = 0, recycle: bool = False):
    """log::Writer::AddRecord's fragmentation of records (host sizes).
    Returns (fragments ctypes array, output bytes, new block_offset)."""
    import numpy as np
    offs = np.ascontiguousarray(np.asarray(src_offsets, dtype=np.uint64))
    lens = np.ascontiguousarray(np.asarray(lengths, dtype=np.uint32))
    n = ctypes.c_uint64()
    out_bytes = ctypes.c_uint64()
    nbo = ctypes.c_uint32()
    check(lib.mck_wal_plan(offs.ctypes.data, lens.ctypes.data, len(lens), block_offset, 1 if recycle else 0,
                           None, 0, ctypes.addressof(n), ctypes.addressof(out_bytes), ctypes.addressof(nbo)),
          "mck_wal_plan")
    frags = (mck_wal_fragment * max(n.value, 1))()
    check(lib.mck_wal_plan(offs.ctypes.data, lens.ctypes.data, len(lens), block_offset, 1 if recycle else 0,
                           ctypes.addressof(frags), n.value, ctypes.addressof(n), ctypes.addressof(out_bytes),
                           ctypes.addressof(nbo)), "mck_wal_plan")
    return frags, n.value, out_bytes.value, nbo.value


class WalBatchWriter:
    """log::Writer for group commits on the device: AddRecords() appends a
    batch of logical records (a device byte tensor + host offsets/lengths)
    to a device-resident log image, fragmented, framed and CRC'd exactly as
    AddRecord/EmitPhysicalRecord would."""

    def __init__(self, log_number: int = 0, recycle_log_files: bool = False, block_offset: int = 0):
        self.log_number = log_number & 0xFFFFFFFF
        self.recycle = recycle_log_files
        self.block_offset = block_offset

    def AddRecords(self, src, src_offsets, lengths, stream=None):
        """Returns the device uint8 tensor of the bytes the records append."""
        torch = _torch()
        frags, n, nbytes, nbo = wal_plan(src_offsets, lengths, self.block_offset, self.recycle)
        dev = src.device
        d_frags = torch.frombuffer(bytearray(bytes(frags)[:n * ctypes.sizeof(mck_wal_fragment)]),
                                   dtype=torch.uint8).to(dev) if n else torch.empty(0, dtype=torch.uint8,
                                                                                     device=dev)
        crc = _empty(max(n, 1), torch.int32, dev)
        out = torch.zeros(nbytes + 16, dtype=torch.uint8, device=dev)
        check(lib.mck_wal_write_batch(src.data_ptr(), d_frags.data_ptr(), n, self.log_number, crc.data_ptr(),
                                      out.data_ptr(), _stream(stream)), "mck_wal_write_batch")
        self.block_offset = nbo
        return out[:nbytes]


def wal_list_records(wal: bytes, log_number: int = 0):
    """log::Reader::ReadRecord's reassembly plan of a host WAL image:
    (fragments ctypes array, nfrags, record offsets, record lengths,
    buffer bytes)."""
    import numpy as np
    buf = bytes(wal)
    nf, nr, nb = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    check(lib.mck_wal_list_records(buf, len(buf), log_number & 0xFFFFFFFF, None, 0, ctypes.addressof(nf),
                                   None, None, 0, ctypes.addressof(nr), ctypes.addressof(nb)),
          "mck_wal_list_records")
    frags = (mck_wal_fragment * max(nf.value, 1))()
    offs = np.zeros(max(nr.value, 1), dtype=np.uint64)
    lens = np.zeros(max(nr.value, 1), dtype=np.uint32)
    check(lib.mck_wal_list_records(buf, len(buf), log_number & 0xFFFFFFFF, ctypes.addressof(frags), nf.value,
                                   ctypes.addressof(nf), offs.ctypes.data, lens.ctypes.data, nr.value,
                                   ctypes.addressof(nr), ctypes.addressof(nb)), "mck_wal_list_records")
    return frags, nf.value, offs[:nr.value], lens[:nr.value], nb.value


class WALRecoveryMode(enum.IntEnum):
    """include/rocksdb/options.h WALRecoveryMode"""
    kTolerateCorruptedTailRecords = 0
    kAbsoluteConsistency = 1
    kPointInTimeRecovery = 2
    kSkipAnyCorruptedRecords = 3


class mck_wal_report(ctypes.Structure):
    _fields_ = [("offset", ctypes.c_uint64), ("bytes", ctypes.c_uint64), ("reason", ctypes.c_int32),
                ("reserved", ctypes.c_uint32)]


class mck_wal_read_out(ctypes.Structure):
    _fields_ = [("struct_size", ctypes.c_uint64),
                ("frags", ctypes.c_void_p), ("frag_cap", ctypes.c_uint64), ("nfrags", ctypes.c_uint64),
                ("rec_offsets", ctypes.c_void_p), ("rec_lengths", ctypes.c_void_p),
                ("rec_file_offsets", ctypes.c_void_p), ("rec_cap", ctypes.c_uint64),
                ("nrecords", ctypes.c_uint64), ("records_bytes", ctypes.c_uint64),
                ("reports", ctypes.c_void_p), ("report_cap", ctypes.c_uint64), ("nreports", ctypes.c_uint64),
                ("dropped_bytes", ctypes.c_uint64), ("end_offset", ctypes.c_uint64),
                ("compression_type", ctypes.c_uint32), ("reserved", ctypes.c_uint32),
                ("stream", ctypes.c_void_p), ("stream_cap", ctypes.c_uint64), ("nstream", ctypes.c_uint64)]


class WalReadPlan(NamedTuple):
    """What log::Reader returns and reports over a whole log (host side)."""
    frags: object            # ctypes array of mck_wal_fragment
    nfrags: int
    rec_offsets: object      # numpy uint64: record r in the contiguous buffer
    rec_lengths: object      # numpy uint32
    rec_file_offsets: object  # numpy uint64: LastRecordOffset of record r
    records_bytes: int
    reports: list            # [(file offset, dropped bytes, reason text)]
    dropped_bytes: int       # ReportCollector::dropped_bytes_
    message: str             # ReportCollector::message_ ("Corruption: ..." appended)
    end_offset: int
    compression_type: int = 0  # WAL compression (kSetCompressionType; kZSTD = 7), 0 = none
    stream: list = []        # compressed logs: [(file offset, length, index in frags or -1)]
                             # of every chunk fed to the reader's StreamingUncompress


def wal_read_records(wal: bytes, log_number: int = 0,
                     recovery_mode: int = WALRecoveryMode.kTolerateCorruptedTailRecords,
                     verified=None) -> WalReadPlan:
    """log::Reader::ReadRecord until false (db/log_reader.cc:69-584) over a
    host WAL image; ``verified`` = the per-block results of
    mck_wal_verify_batch for the same image (numpy int32 [nblocks, 4] or a
    tensor), None = trust every CRC."""
    import numpy as np
    buf = bytes(wal)
    ver = None
    if verified is not None:
        v = verified.cpu().numpy() if hasattr(verified, "cpu") else np.asarray(verified)
        ver = np.ascontiguousarray(v.astype(np.int32).reshape(-1, 4))
    o = mck_wal_read_out()
    o.struct_size = ctypes.sizeof(mck_wal_read_out)
    vp = ver.ctypes.data if ver is not None else None
    check(lib.mck_wal_read_records(buf, len(buf), log_number & 0xFFFFFFFF, int(recovery_mode), vp,
                                   ctypes.addressof(o)), "mck_wal_read_records")
    frags = (mck_wal_fragment * max(o.nfrags, 1))()
    offs = np.zeros(max(o.nrecords, 1), dtype=np.uint64)
    lens = np.zeros(max(o.nrecords, 1), dtype=np.uint32)
    foffs = np.zeros(max(o.nrecords, 1), dtype=np.uint64)
    reps = (mck_wal_report * max(o.nreports, 1))()
    strm = (mck_wal_fragment * max(o.nstream, 1))()
    o2 = mck_wal_read_out(ctypes.sizeof(mck_wal_read_out), ctypes.addressof(frags), o.nfrags, 0, offs.ctypes.data, lens.ctypes.data,
                          foffs.ctypes.data, o.nrecords, 0, 0, ctypes.addressof(reps), o.nreports)
    o2.stream = ctypes.addressof(strm)
    o2.stream_cap = o.nstream
    check(lib.mck_wal_read_records(buf, len(buf), log_number & 0xFFFFFFFF, int(recovery_mode), vp,
                                   ctypes.addressof(o2)), "mck_wal_read_records")
    reports = [(r.offset, r.bytes, lib.mck_wal_reason_string(r.reason).decode()) for r in reps[:o2.nreports]]
    stream = [(f.src_off, f.length, -1 if f.dst_off == 0xFFFFFFFFFFFFFFFF else f.dst_off)
              for f in strm[:o2.nstream]]
    return WalReadPlan(frags, o2.nfrags, offs[:o2.nrecords], lens[:o2.nrecords], foffs[:o2.nrecords],
                       o2.records_bytes, reports, o2.dropped_bytes,
                       "".join("Corruption: " + r[2] for r in reports), o2.end_offset,
                       o2.compression_type, stream)


class mck_wal_recovery_info(ctypes.Structure):
    _fields_ = [("nrecords", ctypes.c_uint64), ("in_place", ctypes.c_uint64), ("gathered", ctypes.c_uint64),
                ("gathered_bytes", ctypes.c_uint64), ("host_walks", ctypes.c_uint32),
                ("has_checksums", ctypes.c_uint32), ("walk_seconds", ctypes.c_double),
                ("device_seconds", ctypes.c_double)]


class WalRecovery(NamedTuple):
    records: object          # device uint8 tensor of every record back to back (gather=True), else None
    rec_offsets: object      # numpy uint64: record r in that (contiguous) record buffer
    rec_lengths: object
    rec_file_offsets: object
    record_checksums: object  # numpy uint64 XXH3_64bits of every record (None: compressed log)
    blocks: object           # per-block device verdicts (mck_wal_block_result as int32 [nblocks, 4])
    reports: list
    dropped_bytes: int
    message: str
    compression_type: int = 0  # compressed WAL: records are compressed chunks (see WalReadPlan)
    stream: list = []
    frags: object = None     # ctypes array of mck_wal_fragment (src_off in the image, dst_off in the buffer)
    nfrags: int = 0
    image: bytes = b""       # the host image (Records() reassembles from it)
    info: object = None      # mck_wal_recovery_info

    def Records(self):
        """The records as bytes (what ReadRecord's *record holds, in order)."""
        if self.records is not None:
            host = bytes(self.records.cpu().numpy().tobytes())
            return [host[int(o):int(o) + int(n)] for o, n in zip(self.rec_offsets, self.rec_lengths)]
        buf = bytearray(sum(int(n) for n in self.rec_lengths) + 1)
        for f in self.frags[:self.nfrags]:
            buf[f.dst_off:f.dst_off + f.length] = self.image[f.src_off:f.src_off + f.length]
        return [bytes(buf[int(o):int(o) + int(n)]) for o, n in zip(self.rec_offsets, self.rec_lengths)]


def WalRecover(wal: bytes, log_number: int = 0,
               recovery_mode: int = WALRecoveryMode.kTolerateCorruptedTailRecords,
               device=None, stream=None, checksum: bool = True, gather: bool = False,
               wal_dev=None) -> WalRecovery:
    """DBImpl::RecoverLogFiles' reader loop (db/db_impl/db_impl_open.cc
    :1204-1221: ReadRecord(&record, &scratch, mode, &record_checksum) until
    false) through ONE entry point, mck_wal_recover: every physical record's
    CRC32C and every single-fragment record's XXH3 record_checksum in one
    device pass over the image (mck_wal_recover_batch), multi-fragment
    records gathered and hashed on the same stream, the reader's walk on the
    host over the verdicts (records, drops and reports of the given
    WALRecoveryMode).  ``wal_dev``: the image already in device memory (a
    uint8 tensor of at least len(wal) + 16 bytes); else it is uploaded.
    ``gather``: also reassemble the records into one device buffer
    (``records``).  ``checksum=False``: the host walk alone, every CRC
    trusted (mck_wal_read_records without verdicts)."""
    import numpy as np
    torch = _torch()
    dev = torch.device("cuda") if device is None else device
    st = stream if stream is not None else torch.cuda.current_stream(dev)
    wal = bytes(wal)
    if not checksum:
        plan = wal_read_records(wal, log_number, recovery_mode, None)
        return WalRecovery(None, plan.rec_offsets, plan.rec_lengths, plan.rec_file_offsets, None, None,
                           plan.reports, plan.dropped_bytes, plan.message, plan.compression_type, plan.stream,
                           plan.frags, plan.nfrags, wal, None)
    with torch.cuda.stream(st):
        img = wal_dev if wal_dev is not None else \
            torch.frombuffer(bytearray(wal + bytes(64)), dtype=torch.uint8).to(dev)
        h = ctypes.c_void_p()
        check(lib.mck_wal_recover(wal, img.data_ptr(), len(wal), log_number & 0xFFFFFFFF, int(recovery_mode),
                                  _stream(st), ctypes.byref(h)), "mck_wal_recover")
        try:
            o = mck_wal_read_out()
            o.struct_size = ctypes.sizeof(mck_wal_read_out)
            check(lib.mck_wal_recovery_read_out(h, ctypes.addressof(o)), "mck_wal_recovery_read_out")
            frags = (mck_wal_fragment * max(o.nfrags, 1))()
            offs = np.zeros(max(o.nrecords, 1), dtype=np.uint64)
            lens = np.zeros(max(o.nrecords, 1), dtype=np.uint32)
            foffs = np.zeros(max(o.nrecords, 1), dtype=np.uint64)
            reps = (mck_wal_report * max(o.nreports, 1))()
            strm = (mck_wal_fragment * max(o.nstream, 1))()
            o2 = mck_wal_read_out(ctypes.sizeof(mck_wal_read_out), ctypes.addressof(frags), o.nfrags, 0,
                                  offs.ctypes.data, lens.ctypes.data, foffs.ctypes.data, o.nrecords, 0, 0,
                                  ctypes.addressof(reps), o.nreports)
            o2.stream = ctypes.addressof(strm)
            o2.stream_cap = o.nstream
            check(lib.mck_wal_recovery_read_out(h, ctypes.addressof(o2)), "mck_wal_recovery_read_out")
            info = mck_wal_recovery_info()
            check(lib.mck_wal_recovery_get_info(h, ctypes.addressof(info)), "mck_wal_recovery_get_info")
            x3 = None
            if info.has_checksums:
                x3 = np.zeros(max(o2.nrecords, 1), dtype=np.uint64)
                check(lib.mck_wal_recovery_checksums(h, x3.ctypes.data, len(x3)), "mck_wal_recovery_checksums")
                x3 = x3[:o2.nrecords]
            nblocks = (len(wal) + 32767) // 32768
            blk = np.zeros((max(nblocks, 1), 4), dtype=np.int32)
            check(lib.mck_wal_recovery_block_results(h, blk.ctypes.data, nblocks), "mck_wal_recovery_block_results")
        finally:
            lib.mck_wal_recovery_free(h)
        reports = [(r.offset, r.bytes, lib.mck_wal_reason_string(r.reason).decode()) for r in reps[:o2.nreports]]
        stream_l = [(f.src_off, f.length, -1 if f.dst_off == 0xFFFFFFFFFFFFFFFF else f.dst_off)
                    for f in strm[:o2.nstream]]
        out = None
        if gather:
            out = torch.zeros(o2.records_bytes + 64, dtype=torch.uint8, device=dev)
            if o2.nfrags:
                d_frags = torch.frombuffer(bytearray(bytes(frags)[:o2.nfrags * ctypes.sizeof(mck_wal_fragment)]),
                                           dtype=torch.uint8).to(dev)
                check(lib.mck_wal_gather_batch(img.data_ptr(), d_frags.data_ptr(), o2.nfrags, out.data_ptr(),
                                               _stream(st)), "mck_wal_gather_batch")
            out = out[:o2.records_bytes]
        blocks = torch.from_numpy(blk[:nblocks]) if nblocks else None
    return WalRecovery(out, offs[:o2.nrecords], lens[:o2.nrecords], foffs[:o2.nrecords], x3, blocks, reports,
                       o2.dropped_bytes, "".join("Corruption: " + r[2] for r in reports), o2.compression_type,
                       stream_l, frags, o2.nfrags, wal, info)


def WalReadRecords(wal: bytes, log_number: int = 0, device=None, stream=None):
    """Recovery on the device (kTolerateCorruptedTailRecords): every logical
    record reassembled into one device buffer and its XXH3_64bits record
    checksum; the physical records' CRCs per 32 KiB block.  Returns (records
    uint8 tensor, offsets, lengths, xxh3 uint64 numpy, per-block verify
    results).  See WalRecover for the reports and other recovery modes."""
    r = WalRecover(wal, log_number, device=device, stream=stream, gather=True)
    return r.records, r.rec_offsets, r.rec_lengths, r.record_checksums, r.blocks


class FragmentBufferedReader:
    """log::FragmentBufferedReader (db/log_reader.cc:618-931): reads a WAL
    that is still being written (secondary instances, WAL tailing;
    allow_retry_read).  ``SetFile(image)`` gives the file as written so far
    (it may only grow); ``ReadRecord()`` returns the next record's bytes or
    None when no complete record is available yet (a partly written record
    is kept; call again after the file grew).  The physical records' CRCs:
    ``verify="device"`` runs mck_wal_verify_batch on the blocks that changed
    since the last call (the verdicts a host walk then consumes),
    ``verify=callable(image) -> per-block results`` supplies them (a CPU
    walk in the CPU tests), ``verify=None`` trusts every CRC."""

    def __init__(self, log_number: int = 0, verify="device", device=None, stream=None):
        import numpy as np
        self._np = np
        self.log_number = log_number & 0xFFFFFFFF
        self.verify = verify
        self.device = device
        self.stream = stream
        h = ctypes.c_void_p()
        check(lib.mck_wal_tail_create(self.log_number, ctypes.byref(h)), "mck_wal_tail_create")
        self._h = h
        self._buf = ctypes.create_string_buffer(1)  # host image (capacity grows by doubling)
        self._len = 0
        self._ver = None       # per-block verdicts of a callable verifier
        self._hver = None
        self._dev = None       # device image (capacity grows by doubling)
        self._dver = None      # device per-block verdicts
        self._clean = 0        # blocks [0, _clean) were verified complete

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            lib.mck_wal_tail_destroy(h)
            self._h = None

    def _device_verdicts(self, img: bytes):
        torch = _torch()
        np = self._np
        dev = torch.device("cuda") if self.device is None else self.device
        st = self.stream if self.stream is not None else torch.cuda.current_stream(dev)
        nb = -(-len(img) // 32768)
        with torch.cuda.stream(st):
            need = nb * 32768 + 64
            if self._dev is None or self._dev.numel() < need:
                cap = max(need, 2 * (self._dev.numel() if self._dev is not None else 0), 1 << 20)
                old = self._dev
                self._dev = torch.zeros(cap, dtype=torch.uint8, device=dev)
                ver = torch.zeros((max(nb, cap // 32768), 4), dtype=torch.int32, device=dev)
                if old is not None:
                    self._dev[:old.numel()].copy_(old)
                    ver[:self._dver.shape[0]].copy_(self._dver)
                self._dver = ver
            # upload and re-verify from the first block not yet verified complete
            lo = self._clean
            start = lo * 32768
            if len(img) > start:
                self._dev[start:len(img)].copy_(torch.frombuffer(bytearray(img[start:]), dtype=torch.uint8))
                check(lib.mck_wal_verify_batch(self._dev.data_ptr() + start, len(img) - start, self.log_number,
                                               self._dver[lo:].data_ptr(), _stream(st)), "mck_wal_verify_batch")
            self._clean = len(img) // 32768
            return np.ascontiguousarray(self._dver[:nb].cpu().numpy().astype(np.int32))

    def SetFile(self, image) -> None:
        """The file as written so far.  It only grows: the bytes already
        handed out must not change (checked over the last block before the
        old end, not the whole prefix, so a poll costs the appended bytes)."""
        np = self._np
        img = memoryview(bytes(image) if not isinstance(image, (bytes, bytearray)) else image)
        old = self._len
        n = len(img)
        lo = max(0, old - 32768)
        if n < old or bytes(img[lo:old]) != bytes(self._buf[lo:old]):
            raise ValueError("a WAL file only grows: the bytes already written must not change")
        if n + 1 > len(self._buf):  # the host image: capacity doubles, only the suffix is copied
            buf = ctypes.create_string_buffer(max(n + 1, 2 * len(self._buf), 1 << 16))
            ctypes.memmove(buf, self._buf, old)
            self._buf = buf
        if n > old:
            ctypes.memmove(ctypes.addressof(self._buf) + old, bytes(img[old:n]), n - old)
        self._len = n
        nb = -(-n // 32768)
        if self.verify == "device":
            ver = self._device_verdicts(img) if n else None
        elif callable(self.verify):
            # re-verify from the first block not verified complete (the blocks
            # before it cannot change)
            if self._ver is None or self._ver.shape[0] < nb:
                v = np.zeros((max(nb, 1), 4), np.int32)
                if self._ver is not None:
                    v[:self._ver.shape[0]] = self._ver
                self._ver = v
            c = self._clean
            if n > c * 32768:
                res = np.asarray(self.verify(bytes(img[c * 32768:n])), dtype=np.int64).astype(np.int32)
                self._ver[c:c + len(res)] = res.reshape(-1, 4)
            self._clean = n // 32768
            ver = self._ver if n else None
        else:
            ver = None
        self._hver = ver
        check(lib.mck_wal_tail_set_image(self._h, self._buf, n,
                                         ver.ctypes.data if ver is not None else None), "mck_wal_tail_set_image")

    @property
    def _img(self) -> bytes:
        return self._buf.raw[:self._len]

    def _supply_verdict(self) -> None:
        """MCK_EAGAIN: verify the rest of a block the reader passed a checksum
        failure in (mck_wal_tail_pending_verify) as one block."""
        np = self._np
        off, n = ctypes.c_uint64(), ctypes.c_uint64()
        if not lib.mck_wal_tail_pending_verify(self._h, ctypes.byref(off), ctypes.byref(n)):
            raise RuntimeError("mck_wal_tail_read_record asked for a verdict but none is pending")
        o, k = off.value, n.value
        if self.verify == "device":
            torch = _torch()
            dev = torch.device("cuda") if self.device is None else self.device
            st = self.stream if self.stream is not None else torch.cuda.current_stream(dev)
            with torch.cuda.stream(st):
                res = torch.zeros((1, 4), dtype=torch.int32, device=dev)
                check(lib.mck_wal_verify_batch(self._dev.data_ptr() + o, k, self.log_number, res.data_ptr(),
                                               _stream(st)), "mck_wal_verify_batch")
                r = np.ascontiguousarray(res.cpu().numpy().astype(np.int32))
        else:
            r = np.ascontiguousarray(np.asarray(self.verify(self._buf.raw[o:o + k]), dtype=np.int64)
                                     .astype(np.int32)[:1])
        check(lib.mck_wal_tail_add_verdict(self._h, o, r.ctypes.data), "mck_wal_tail_add_verdict")

    def ReadRecord(self) -> Optional[bytes]:
        nf, nb, lro = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        supplied = set()
        while True:
            rc = lib.mck_wal_tail_read_record(self._h, ctypes.byref(nf), ctypes.byref(nb), ctypes.byref(lro))
            if rc != MCK_EAGAIN:
                break
            off = ctypes.c_uint64()
            lib.mck_wal_tail_pending_verify(self._h, ctypes.byref(off), None)
            if off.value in supplied:  # the verdict added did not decide it: never spin
                raise RuntimeError(f"WAL tail reader: the verdict for offset {off.value} did not resolve it")
            supplied.add(off.value)
            self._supply_verdict()
        if rc < 0:
            check(rc, "mck_wal_tail_read_record")
        if rc == 0:
            return None
        frags = (mck_wal_fragment * max(nf.value, 1))()
        check(lib.mck_wal_tail_record_fragments(self._h, ctypes.addressof(frags), nf.value),
              "mck_wal_tail_record_fragments")
        self.last_record_offset = lro.value
        out = bytearray(nb.value)
        raw = self._buf
        for f in frags[:nf.value]:
            out[f.dst_off:f.dst_off + f.length] = ctypes.string_at(ctypes.addressof(raw) + f.src_off, f.length)
        return bytes(out)

    def OldRecordOffset(self) -> Optional[int]:
        """The header offset of an older log instance's record the reader is
        stopped at (it returns "no record" there forever, where the
        reference's FragmentBufferedReader would re-parse the same header
        without end), or None."""
        off = ctypes.c_uint64()
        return off.value if lib.mck_wal_tail_old_record(self._h, ctypes.byref(off)) else None

    def LastRecordOffset(self) -> int:
        return getattr(self, "last_record_offset", 0)

    def UnmarkEOF(self) -> None:
        check(lib.mck_wal_tail_unmark_eof(self._h), "mck_wal_tail_unmark_eof")

    def IsEOF(self) -> bool:
        return bool(lib.mck_wal_tail_is_eof(self._h))

    def _reports(self):
        n, dropped = ctypes.c_uint64(), ctypes.c_uint64()
        check(lib.mck_wal_tail_reports(self._h, None, 0, ctypes.byref(n), ctypes.byref(dropped)), "reports")
        reps = (mck_wal_report * max(n.value, 1))()
        check(lib.mck_wal_tail_reports(self._h, ctypes.addressof(reps), n.value, ctypes.byref(n),
                                       ctypes.byref(dropped)), "reports")
        return [(r.offset, r.bytes, lib.mck_wal_reason_string(r.reason).decode()) for r in reps[:n.value]], \
            dropped.value

    @property
    def dropped_bytes(self) -> int:
        return self._reports()[1]

    @property
    def message(self) -> str:
        """ReportCollector::message_: "Corruption: <reason>" per report."""
        return "".join("Corruption: " + r[2] for r in self._reports()[0])


__all__ += ["wal_plan", "WalBatchWriter", "mck_wal_fragment", "wal_list_records", "WalReadRecords",
            "WALRecoveryMode", "wal_read_records", "WalReadPlan", "WalRecover", "WalRecovery",
            "FragmentBufferedReader", "wal_recover_batch", "wal_plan_records", "mck_wal_recovery_info"]


# ---------------------------------------------------------------------------
# host-resident batches (mck_host_batch_checksum): the copy-inclusive path
# ---------------------------------------------------------------------------

def host_batch_checksum(kind: int, host, offsets=None, lengths=None, stride: int = 0, length: int = 0,
                        count: Optional[int] = None, mask: bool = False, ndev: int = 0,
                        chunk_bytes: int = 0):
    """Checksum spans that live in HOST memory (pinned gives the full PCIe
    rate): H2D in double-buffered chunks, CRC32C (``kind`` =
    ChecksumType.kCRC32c, optionally masked) or XXH3_64bits (kXXH3) on the
    device, results back to the host.  ``host``: a numpy uint8 array, a CPU
    torch uint8 tensor (pinned or not) or bytes; offsets/lengths: host
    sequences (None = uniform stride/length).  ndev <= 0: the current device;
    otherwise devices [0, ndev).  Returns (numpy results, seconds)."""
    import numpy as np
    if isinstance(host, (bytes, bytearray, memoryview)):
        host = np.frombuffer(bytes(host), dtype=np.uint8)
    base = host.data_ptr() if hasattr(host, "data_ptr") else host.ctypes.data
    offs = None if offsets is None else np.ascontiguousarray(np.asarray(offsets, dtype=np.uint64))
    lens = None if lengths is None else np.ascontiguousarray(np.asarray(lengths, dtype=np.uint32))
    if count is None:
        count = len(offs) if offs is not None else len(lens) if lens is not None else 0
    out = np.zeros(count, dtype=np.uint64 if kind == ChecksumType.kXXH3 else np.uint32)
    secs = ctypes.c_double()
    o32 = out.ctypes.data if kind != ChecksumType.kXXH3 else None
    o64 = out.ctypes.data if kind == ChecksumType.kXXH3 else None
    check(lib.mck_host_batch_checksum(int(kind), base, None if offs is None else offs.ctypes.data,
                                      None if lens is None else lens.ctypes.data, stride, length, count,
                                      1 if mask else 0, ndev, chunk_bytes, o32, o64, ctypes.byref(secs)),
          "mck_host_batch_checksum")
    return out, secs.value


__all__ += ["host_batch_checksum"]


# ---------------------------------------------------------------------------
# statistics (include/rocksdb/statistics.h tickers of this path)
# ---------------------------------------------------------------------------

class mck_statistics(ctypes.Structure):
    _fields_ = [("block_checksum_compute_count", ctypes.c_uint64),
                ("block_checksum_mismatch_count", ctypes.c_uint64), ("batches", ctypes.c_uint64),
                ("spans", ctypes.c_uint64), ("bytes_known", ctypes.c_uint64)]


def statistics(reset: bool = False) -> dict:
    """The engine's counters: BLOCK_CHECKSUM_COMPUTE_COUNT /
    BLOCK_CHECKSUM_MISMATCH_COUNT (statistics.h:451,455; the mismatches are
    counted on the device -- synchronise first), batches, spans and the
    bytes of batches with host-known lengths.  reset=True zeroes them."""
    s = mck_statistics()
    check(lib.mck_statistics_get(ctypes.addressof(s), 1 if reset else 0), "mck_statistics_get")
    return {"BLOCK_CHECKSUM_COMPUTE_COUNT": s.block_checksum_compute_count,
            "BLOCK_CHECKSUM_MISMATCH_COUNT": s.block_checksum_mismatch_count,
            "batches": s.batches, "spans": s.spans, "bytes_known": s.bytes_known}


__all__ += ["statistics"]


# ---------------------------------------------------------------------------
# PerfContext: block_checksum_time (include/rocksdb/perf_context.h:97,
# table/block_based/reader_common.cc:29), per thread
# ---------------------------------------------------------------------------

class PerfLevel(enum.IntEnum):
    """include/rocksdb/perf_level.h"""
    kDisable = 1
    kEnableCount = 2
    kEnableTimeExceptForMutex = 3
    kEnableTimeAndCPUTimeExceptForMutex = 4
    kEnableTime = 5


class mck_perf_context(ctypes.Structure):
    _fields_ = [("block_checksum_time", ctypes.c_uint64), ("block_checksum_count", ctypes.c_uint64),
                ("block_checksum_batches", ctypes.c_uint64)]


def SetPerfLevel(level: int) -> None:
    check(lib.mck_set_perf_level(int(level)), "mck_set_perf_level")


def GetPerfLevel() -> PerfLevel:
    return PerfLevel(lib.mck_get_perf_level())


def get_perf_context(reset: bool = False) -> dict:
    """This thread's perf context: block_checksum_time = nanoseconds of DEVICE
    time of the VerifyBlockChecksum batches it issued at a timing level
    (waits for them), block_checksum_count = blocks verified, batches."""
    c = mck_perf_context()
    check(lib.mck_perf_context_get(ctypes.addressof(c), 1 if reset else 0), "mck_perf_context_get")
    return {"block_checksum_time": c.block_checksum_time, "block_checksum_count": c.block_checksum_count,
            "block_checksum_batches": c.block_checksum_batches}


__all__ += ["PerfLevel", "SetPerfLevel", "GetPerfLevel", "get_perf_context"]

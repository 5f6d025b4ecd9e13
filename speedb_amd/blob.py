"""Blob files (db/blob/blob_log_format.{h,cc}): the host
walks the file's header / records / footer (mck_blob_list_records), and the
records' header and blob CRCs are checked -- or, on the write side,
computed and stored -- on the GPU in one batch (mck_blob_record_batch).

Mirrors BlobLogSequentialReader + BlobLogRecord::DecodeHeaderFrom /
CheckBlobCRC (read) and BlobLogRecord::EncodeHeaderTo (write), with the
reference's Status messages.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import List, Optional, Tuple

import numpy as np

from ._lib import check, lib
from .checksum import Status, _stream, crc32c

HEADER_SIZE, FOOTER_SIZE, RECORD_HEADER_SIZE = 30, 32, 32
MAGIC = 2395959


class mck_blob_file_info(ctypes.Structure):
    _fields_ = [("version", ctypes.c_uint32), ("column_family_id", ctypes.c_uint32),
                ("has_ttl", ctypes.c_uint8), ("compression", ctypes.c_uint8),
                ("has_footer", ctypes.c_uint8), ("reserved", ctypes.c_uint8),
                ("expiration_first", ctypes.c_uint64), ("expiration_second", ctypes.c_uint64),
                ("footer_blob_count", ctypes.c_uint64), ("footer_crc", ctypes.c_uint32),
                ("reserved2", ctypes.c_uint32)]


class mck_blob_record(ctypes.Structure):
    _fields_ = [("offset", ctypes.c_uint64), ("key_size", ctypes.c_uint64),
                ("value_size", ctypes.c_uint64)]


@dataclass
class BlobRecord:
    offset: int
    key_size: int
    value_size: int


class BlobError(RuntimeError):
    def __init__(self, rc: int, msg: str):
        super().__init__(msg)
        self.rc = rc
        self.status = Status("Corruption" if rc == -5 else "Not implemented" if rc == -6
                             else "Invalid argument", msg)


def list_records(image: bytes) -> Tuple[mck_blob_file_info, List[BlobRecord]]:
    buf = bytes(image)
    info = mck_blob_file_info()
    n = ctypes.c_uint64()
    rc = lib.mck_blob_list_records(buf, len(buf), ctypes.addressof(info), None, 0, ctypes.addressof(n))
    if rc:
        raise BlobError(rc, lib.mck_last_error().decode(errors="replace"))
    arr = (mck_blob_record * max(n.value, 1))()
    rc = lib.mck_blob_list_records(buf, len(buf), ctypes.addressof(info), ctypes.addressof(arr), n.value,
                                   ctypes.addressof(n))
    if rc:
        raise BlobError(rc, lib.mck_last_error().decode(errors="replace"))
    return info, [BlobRecord(int(r.offset), int(r.key_size), int(r.value_size)) for r in arr[:n.value]]


def record_batch(write: bool, dev_file, offsets, lengths, status=None, count=None, stream=None):
    """The device batch over records (offsets: int64 tensor of header
    offsets, lengths: int32 tensor of key_size + value_size)."""
    import torch
    n = offsets.numel()
    if not write and status is None:
        status = torch.empty(n, dtype=torch.uint8, device=dev_file.device)
    check(lib.mck_blob_record_batch(1 if write else 0, dev_file.data_ptr(), offsets.data_ptr(),
                                    lengths.data_ptr(), n, None if write else status.data_ptr(),
                                    None if count is None else count.data_ptr(), _stream(stream)),
          "mck_blob_record_batch")
    return status


def _device_records(image, recs, device):
    import torch
    dev = torch.frombuffer(bytearray(bytes(image) + bytes(64)), dtype=torch.uint8).to(device)
    offs = torch.tensor([r.offset for r in recs], dtype=torch.int64, device=device)
    lens = torch.tensor([r.key_size + r.value_size for r in recs], dtype=torch.int32, device=device)
    return dev, offs, lens


def VerifyBlobFile(image: bytes, device=None, stream=None, per_record: Optional[list] = None) -> Status:
    """Every record's header CRC and blob CRC in one GPU batch, plus the
    footer CRC.  First failure as the reference's Status."""
    import torch
    try:
        info, recs = list_records(image)
    except BlobError as e:
        return e.status
    if info.has_footer:
        foot = bytes(image[-FOOTER_SIZE:])
        if crc32c.Mask(crc32c.Value(foot[:FOOTER_SIZE - 4])) != info.footer_crc:
            return Status.Corruption("Error while decoding blob log footer: CRC mismatch")
    if not recs:
        return Status.OK()
    device = torch.device("cuda") if device is None else device
    dev, offs, lens = _device_records(image, recs, device)
    st = record_batch(False, dev, offs, lens, stream=stream).cpu().numpy()
    first = Status.OK()
    for r, s in zip(recs, st.tolist()):
        cur = Status.OK()
        if s & 1:  # blob_log_format.cc:129 (DecodeHeaderFrom)
            cur = Status.Corruption("Error while decoding blob record: Header CRC mismatch")
        elif s & 2:  # blob_log_format.cc:140 (CheckBlobCRC)
            cur = Status.Corruption("Blob CRC mismatch")
        if first.ok() and not cur.ok():
            first = cur
        if per_record is not None:
            per_record.append((r, cur))
    return first


def WriteRecordCrcs(dev_file, offsets, lengths, stream=None) -> None:
    """BlobLogRecord::EncodeHeaderTo's CRC fields for every record of a
    device-resident blob file image whose headers hold the sizes."""
    record_batch(True, dev_file, offsets, lengths, stream=stream)


__all__ = ["list_records", "record_batch", "VerifyBlobFile", "WriteRecordCrcs", "BlobRecord", "BlobError"]

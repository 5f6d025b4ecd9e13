"""WritableFileWriter checksum handoff:
file/writable_file_writer.{h,cc} with perform_data_verification_ on
(checksum handoff for the file type, options.checksum_handoff_file_types) and
buffered, non-direct I/O, no rate limiter.

The writer hands every FSWritableFile::Append a DataVerificationInfo whose
checksum is the CRC32C of the bytes written:

* WriteBuffered (:544-636): Crc32cHandoffChecksumCalculation (:743-747) =
  EncodeFixed32(crc32c::Extend(0, data));
* WriteBufferedWithChecksum (:638-720, buffered_data_with_checksum_): the
  running buffered_data_crc32c_checksum_, kept by Append (:44-175) with
  crc32c::Crc32cCombine over caller-supplied checksums (the WAL writer passes
  each payload's CRC, db/log_writer.cc) and crc32c::Extend over the rest.

Here the bytes are device-resident (torch uint8 tensors: e.g. the device WAL
writer's log stream) and every CRC the reference computes over data -- Extend,
Value, Crc32cHandoffChecksumCalculation -- is deferred and computed on the GPU
in ONE batch (mck_handoff_checksum_batch) when the writes are resolved; the
u32 algebra (Combine) stays on the host, as in the reference.  ``writes``
lists what the file receives: (offset, size, checksum or None).
"""
from __future__ import annotations

import ctypes
from typing import Callable, List, Optional, Sequence, Tuple

from ._lib import check, lib
from .checksum import Spans, _stream, _torch, crc32c

# a CRC term of a running checksum: a known u32, or a device piece to hash
Piece = Tuple[object, int, int]  # (uint8 tensor, start, length)


def handoff_checksum_batch(pieces: Sequence[Piece], stream=None) -> List[int]:
    """crc32c::Extend(0, piece) of every (tensor, start, length) piece on the
    GPU, one batch per base tensor."""
    torch = _torch()
    out: List[Optional[int]] = [None] * len(pieces)
    by_base = {}
    for i, (t, s, n) in enumerate(pieces):
        by_base.setdefault(id(t), (t, []))[1].append((i, s, n))
    for t, items in by_base.values():
        dev = t.device
        st = stream if stream is not None else torch.cuda.current_stream(dev)
        # descriptors, kernel and readback all on `st`: .cpu() inside the
        # context waits for that stream, not for whatever stream is current
        with torch.cuda.stream(st):
            offs = torch.tensor([s for _, s, _ in items], dtype=torch.int64, device=dev)
            lens = torch.tensor([n for _, _, n in items], dtype=torch.int32, device=dev)
            res = torch.empty(len(items), dtype=torch.int32, device=dev)
            sp = Spans(t, len(items), offs, lens).c()
            check(lib.mck_handoff_checksum_batch(ctypes.byref(sp), res.data_ptr(), _stream(st)),
                  "mck_handoff_checksum_batch")
            vals = res.cpu().tolist()
        for (i, _, _), v in zip(items, vals):
            out[i] = v & 0xFFFFFFFF
    return out  # type: ignore[return-value]


class _Sum:
    """A running CRC as terms folded with Crc32cCombine: (crc, len) known
    values and pieces whose Value is computed later."""

    def __init__(self):
        self.terms: List[tuple] = []

    def reset(self, terms=None):
        self.terms = list(terms or [])

    def combine(self, crc: int, n: int):   # Crc32cCombine(sum, crc, n)
        self.terms.append(("crc", crc, n))

    def extend(self, piece: Piece):        # Extend(sum, data) = Combine(sum, Value(data), n)
        self.terms.append(("piece", piece))


class WritableFileWriter:
    """Buffered WritableFileWriter with checksum handoff.  ``crc_batch`` maps
    pieces to their crc32c::Value (default: the GPU batch)."""

    def __init__(self, max_buffer_size: int = 1 << 20, buffered_data_with_checksum: bool = False,
                 perform_data_verification: bool = True,
                 crc_batch: Optional[Callable[[Sequence[Piece]], List[int]]] = None):
        self.max_buffer_size = max_buffer_size
        self.cap = min(65536, max_buffer_size)  # writable_file_writer.h ctor
        self.bdwc = buffered_data_with_checksum
        self.pdv = perform_data_verification
        self.crc_batch = crc_batch or handoff_checksum_batch
        self.buf: List[Piece] = []
        self.size = 0
        self.buffered = _Sum()
        self.filesize = 0
        self._flushed = 0
        self._pending: List[tuple] = []  # (offset, size, checksum terms or None)

    # -- buffer -------------------------------------------------------------
    def _buf_append(self, t, s, n) -> int:
        k = min(n, self.cap - self.size)
        if k:
            self.buf.append((t, s, k))
            self.size += k
        return k

    def _write(self, pieces: List[Piece], terms: Optional[list]):
        n = sum(p[2] for p in pieces)
        self._pending.append((self._flushed, n, terms, pieces))
        self._flushed += n

    def _write_buffered(self, pieces: List[Piece]):
        # :544-636: one Append per rate-limiter grant (no limiter: all of it),
        # checksum = Crc32cHandoffChecksumCalculation(src, allowed)
        self._write(pieces, [("piece", p) for p in pieces] if self.pdv else None)

    def _write_buffered_with_checksum(self, pieces: List[Piece]):
        # :638-720: checksum = buffered_data_crc32c_checksum_, then reset
        self._write(pieces, list(self.buffered.terms))
        self.buffered.reset()

    # -- reference API --------------------------------------------------------
    def Append(self, data, crc32c_checksum: int = 0, start: int = 0, length: Optional[int] = None):
        """:44-175.  ``data``: device uint8 tensor (bytes [start, start+length)).
        The bytes are copied at Append time (the reference copies them into
        buf_, or writes them out, before Append returns), so the caller may
        reuse its tensor at once: every deferred checksum is over the bytes
        as they were appended."""
        n = data.numel() - start if length is None else length
        if n > 0:
            data, start = data[start:start + n].clone(), 0  # device-to-device snapshot
        left, src = n, start
        if self.cap - self.size < left:  # :68-82 grow the buffer
            cap = self.cap
            while cap < self.max_buffer_size:
                desired = min(cap * 2, self.max_buffer_size)
                if desired - self.size >= left:
                    self.cap = desired
                    break
                cap *= 2
        if self.cap - self.size < left and self.size > 0:  # :85-97
            self.Flush()
        if self.pdv and self.bdwc and crc32c_checksum != 0:  # :99-131
            if self.cap - self.size >= left:
                self._buf_append(data, src, left)
                self.buffered.combine(crc32c_checksum, left)
            else:
                assert self.size == 0
                self.buffered.reset([("crc", crc32c_checksum, left)])
                self._write_buffered_with_checksum([(data, src, left)])
        else:  # :132-165
            if self.cap >= left:
                while left > 0:
                    k = self._buf_append(data, src, left)
                    if self.pdv and self.bdwc:
                        self.buffered.extend((data, src, k))
                    left -= k
                    src += k
                    if left > 0:
                        self.Flush()
            else:
                assert self.size == 0
                if self.pdv and self.bdwc:
                    self.buffered.reset([("piece", (data, src, left))])
                    self._write_buffered_with_checksum([(data, src, left)])
                else:
                    self._write_buffered([(data, src, left)])
        self.filesize += n

    def Flush(self):
        """:325-360: write the buffer out (WriteBuffered[WithChecksum])."""
        if self.size > 0:
            pieces = self.buf
            if self.pdv and self.bdwc:
                self._write_buffered_with_checksum(pieces)
            else:
                self._write_buffered(pieces)
            self.buf, self.size = [], 0

    def Close(self):
        self.Flush()

    def GetFileSize(self) -> int:
        return self.filesize

    # -- the file's view ------------------------------------------------------
    @property
    def writes(self) -> List[Tuple[int, int, Optional[int]]]:
        """(offset, size, handoff checksum u32 or None) of every
        FSWritableFile::Append so far; all pending data CRCs in one batch."""
        need = [t[1] for _, _, terms, _ in self._pending if terms for t in terms if t[0] == "piece"]
        vals = iter(self.crc_batch(need) if need else [])
        out = []
        for off, size, terms, _ in self._pending:
            if terms is None:
                out.append((off, size, None))
                continue
            c = 0
            for t in terms:
                if t[0] == "crc":
                    c = crc32c.Crc32cCombine(c, t[1], t[2])
                else:
                    c = crc32c.Crc32cCombine(c, next(vals), t[1][2])
            out.append((off, size, c))
        return out

    def written_pieces(self) -> List[List[Piece]]:
        return [p for _, _, _, p in self._pending]

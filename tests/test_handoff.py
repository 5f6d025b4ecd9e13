"""WritableFileWriter checksum handoff (SURVEY.md 8f row 2,
file/writable_file_writer.cc:44-175 Append, :325-360 Flush, :544-720
WriteBuffered[WithChecksum], :743-747 Crc32cHandoffChecksumCalculation).

RefWriter below restates the reference's buffering over host bytes with the
oracle's CRC32C computed eagerly, exactly where the reference calls Extend /
Value / Crc32cCombine; speedb_amd.handoff.WritableFileWriter defers every data
CRC into one device batch and folds with Combine.  Both must hand the file
the same (offset, size, checksum) sequence, and every checksum must be
Value() of the bytes it covers.
"""
import random

import pytest


class RefWriter:
    def __init__(self, oracle, max_buffer_size, bdwc, pdv=True):
        self.o, self.max, self.bdwc, self.pdv = oracle, max_buffer_size, bdwc, pdv
        self.cap = min(65536, max_buffer_size)
        self.buf = b""
        self.bck = 0  # buffered_data_crc32c_checksum_
        self.writes, self.off = [], 0

    def _wb(self, data):  # WriteBuffered
        self.writes.append((self.off, len(data), self.o.Extend(0, data) if self.pdv else None))
        self.off += len(data)

    def _wbc(self, data):  # WriteBufferedWithChecksum
        self.writes.append((self.off, len(data), self.bck))
        self.off += len(data)
        self.bck = 0

    def Flush(self):
        if self.buf:
            (self._wbc if (self.pdv and self.bdwc) else self._wb)(self.buf)
            self.buf = b""

    def Append(self, data, crc=0):
        left = len(data)
        if self.cap - len(self.buf) < left:
            cap = self.cap
            while cap < self.max:
                desired = min(cap * 2, self.max)
                if desired - len(self.buf) >= left:
                    self.cap = desired
                    break
                cap *= 2
        if self.cap - len(self.buf) < left and self.buf:
            self.Flush()
        if self.pdv and self.bdwc and crc != 0:
            if self.cap - len(self.buf) >= left:
                self.buf += data
                self.bck = self.o.Combine(self.bck, crc, left)
            else:
                self.bck = crc
                self._wbc(data)
        elif self.cap >= left:
            src = data
            while src:
                k = min(len(src), self.cap - len(self.buf))
                self.buf += src[:k]
                if self.pdv and self.bdwc:
                    self.bck = self.o.Extend(self.bck, src[:k])
                src = src[k:]
                if src:
                    self.Flush()
        else:
            if self.pdv and self.bdwc:
                self.bck = self.o.Value(data)
                self._wbc(data)
            else:
                self._wb(data)


def _workload(rnd, oracle, n=60):
    """(bytes, crc passed or 0): WAL-like header/payload pairs, big blobs."""
    out = []
    for _ in range(n):
        kind = rnd.random()
        if kind < 0.4:
            out.append((bytes(rnd.getrandbits(8) for _ in range(7)), 0))  # record header
            p = bytes(rnd.getrandbits(8) for _ in range(rnd.randrange(1, 3000)))
            out.append((p, oracle.Value(p)))                              # payload + its CRC
        elif kind < 0.8:
            out.append((bytes(rnd.getrandbits(8) for _ in range(rnd.randrange(1, 40000))), 0))
        else:
            p = bytes(rnd.getrandbits(8) for _ in range(rnd.randrange(60000, 300000)))
            out.append((p, oracle.Value(p) if rnd.random() < 0.5 else 0))
    return out


def _run(torch, device, oracle, crc_batch, rnd, max_buf, bdwc, pdv=True):
    from speedb_amd.handoff import WritableFileWriter
    items = _workload(rnd, oracle)
    ref = RefWriter(oracle, max_buf, bdwc, pdv)
    w = WritableFileWriter(max_buf, bdwc, pdv, crc_batch=crc_batch)
    stream = b"".join(d for d, _ in items)
    dev = torch.frombuffer(bytearray(stream + bytes(16)), dtype=torch.uint8).to(device)
    pos = 0
    for d, c in items:
        ref.Append(d, c)
        w.Append(dev, c, start=pos, length=len(d))
        pos += len(d)
    ref.Flush()
    w.Close()
    got = w.writes
    assert got == ref.writes
    assert sum(s for _, s, _ in got) == len(stream) == w.GetFileSize()
    for off, size, ck in got:  # every handoff checksum is Value() of its bytes
        if pdv:
            assert ck == oracle.Value(stream[off:off + size])
        else:
            assert ck is None


@pytest.mark.parametrize("max_buf,bdwc,pdv", [(1 << 20, False, True), (1 << 20, True, True),
                                              (65536, True, True), (200000, True, True),
                                              (1 << 20, False, False)])
def test_handoff_bookkeeping_cpu(oracle, max_buf, bdwc, pdv):
    """Host bookkeeping with the oracle as the CRC provider (no GPU)."""
    torch = pytest.importorskip("torch")

    def crc_batch(pieces):
        return [oracle.Value(bytes(t[s:s + n].numpy().tobytes())) for t, s, n in pieces]
    _run(torch, "cpu", oracle, crc_batch, random.Random(max_buf + bdwc), max_buf, bdwc, pdv)


@pytest.mark.gpu
@pytest.mark.parametrize("max_buf,bdwc", [(1 << 20, False), (1 << 20, True), (65536, True)])
def test_handoff_gpu(gpu, oracle, max_buf, bdwc):
    """The deferred data CRCs on the GPU (mck_handoff_checksum_batch)."""
    _run(gpu, "cuda", oracle, None, random.Random(7 + max_buf + bdwc), max_buf, bdwc)


@pytest.mark.gpu
def test_handoff_checksum_batch_is_encode_fixed32(gpu, oracle):
    """out[i] viewed as bytes = EncodeFixed32(crc32c::Extend(0, piece))."""
    import ctypes
    import speedb_amd
    from speedb_amd._lib import lib
    torch = gpu
    rnd = random.Random(3)
    data = bytes(rnd.getrandbits(8) for _ in range(100000))
    d = torch.frombuffer(bytearray(data + bytes(16)), dtype=torch.uint8).cuda()
    cuts = sorted(rnd.sample(range(1, len(data)), 40))
    offs = [0] + cuts
    lens = [b - a for a, b in zip(offs, cuts + [len(data)])]
    sp = speedb_amd.Spans(d, len(offs), torch.tensor(offs, dtype=torch.int64, device="cuda"),
                          torch.tensor(lens, dtype=torch.int32, device="cuda"))
    out = torch.empty(len(offs), dtype=torch.int32, device="cuda")
    assert lib.mck_handoff_checksum_batch(ctypes.byref(sp.c()), out.data_ptr(), None) == 0
    raw = out.cpu().numpy().tobytes()
    for i, (o, n) in enumerate(zip(offs, lens)):
        assert raw[4 * i:4 * i + 4] == oracle.Extend(0, data[o:o + n]).to_bytes(4, "little")


def _run_reused_staging(torch, device, oracle, crc_batch, rnd):
    """Every Append comes from ONE staging tensor that the caller overwrites
    right after the call (a WAL writer reusing its record buffer): the
    handoff checksums must cover the bytes as appended, as the reference's
    copy into buf_ guarantees (writable_file_writer.cc:107-165)."""
    from speedb_amd.handoff import WritableFileWriter
    items = _workload(rnd, oracle, n=30)
    ref = RefWriter(oracle, 1 << 20, True)
    w = WritableFileWriter(1 << 20, True, True, crc_batch=crc_batch)
    stage = torch.zeros(max(len(d) for d, _ in items) + 16, dtype=torch.uint8, device=device)
    for d, c in items:
        stage[:len(d)].copy_(torch.frombuffer(bytearray(d), dtype=torch.uint8))
        ref.Append(d, c)
        w.Append(stage, c, start=0, length=len(d))
        stage.fill_(0xA5)  # the caller reuses its buffer before the writes are resolved
    ref.Flush()
    w.Close()
    assert w.writes == ref.writes


def test_handoff_append_snapshots_bytes_cpu(oracle):
    torch = pytest.importorskip("torch")

    def crc_batch(pieces):
        return [oracle.Value(bytes(t[s:s + n].numpy().tobytes())) for t, s, n in pieces]
    _run_reused_staging(torch, "cpu", oracle, crc_batch, random.Random(41))


@pytest.mark.gpu
def test_handoff_append_snapshots_bytes_gpu(gpu, oracle):
    _run_reused_staging(gpu, "cuda", oracle, None, random.Random(43))


@pytest.mark.gpu
def test_handoff_checksum_batch_side_stream(gpu, oracle):
    """The batch issued on a non-default stream: the readback waits for that
    stream (the kernel is queued behind a long one on it)."""
    from speedb_amd.handoff import handoff_checksum_batch
    torch = gpu
    rnd = random.Random(5)
    data = bytes(rnd.getrandbits(8) for _ in range(300000))
    d = torch.frombuffer(bytearray(data + bytes(16)), dtype=torch.uint8).cuda()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())  # d is uploaded
    big = torch.empty(1 << 28, dtype=torch.uint8, device="cuda")
    with torch.cuda.stream(side):
        for _ in range(8):
            big.fill_(1)  # keeps the side stream busy for a while
    pieces = [(d, o, 9000) for o in range(0, 290000, 9000)]
    got = handoff_checksum_batch(pieces, stream=side)
    assert got == [oracle.Value(data[o:o + 9000]) for _, o, _ in pieces]

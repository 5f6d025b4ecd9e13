"""log::Reader semantics pinned to the reference's own tests: db/log_test.cc
(LogTest, parameterised on recyclable logs) restated as byte-level WAL
fixtures.  Each case writes the records with the test-side restatement of
log::Writer (tests/formats.py WalWriter, log number 123 as in LogTest),
applies the same byte edits (IncrementByte / SetByte / FixChecksum /
ShrinkSize), and asserts what log_test.cc asserts: the records ReadRecord
returns until "EOF", ReportCollector::dropped_bytes_ and the reported
message.  The reader is mck_wal_read_records (host walk) over per-block CRC
verdicts -- from the oracle walk here (CPU), from mck_wal_verify_batch on the
device in the -m gpu leg, which also checks every record's XXH3
record_checksum.  FragmentBufferedReader (allow_retry_read) is restated
below; compressed logs are walked and verified (the decompression is the
caller's, see test_compressed_wal_walk)."""
import struct

import numpy as np
import pytest

from formats import K_BLOCK, K_HEADER, K_RECYCLABLE_HEADER, WalWriter, wal_expected_blocks

LOG = 123
kTolerate, kAbsolute, kPIT, kSkipAny = 0, 1, 2, 3
kFirstType, kMiddleType, kLastType = 2, 3, 4
kRecyclableFirstType, kRecyclableMiddleType, kRecyclableLastType = 6, 7, 8


def big_string(part: str, n: int) -> bytes:  # log_test.cc:23-33
    s = part.encode()
    return (s * (n // len(s) + 1))[:n]


def number_string(i: int) -> bytes:  # log_test.cc:36-40
    return f"{i}.".encode()


class Log:
    """log_test.cc's LogTest fixture over a WalWriter image."""

    def __init__(self, oracle, recycle):
        self.o = oracle
        self.recycle = recycle
        self.hs = K_RECYCLABLE_HEADER if recycle else K_HEADER
        self.w = WalWriter(oracle, log_number=LOG, recycle=recycle)

    def write(self, msg: bytes):
        self.w.add_record(msg)

    def written(self):
        return len(self.w.buf)

    def increment_byte(self, off, delta):
        self.w.buf[off] = (self.w.buf[off] + delta) & 0xFF

    def set_byte(self, off, b):
        self.w.buf[off] = b & 0xFF

    def shrink(self, n):
        del self.w.buf[len(self.w.buf) - n:]

    def fix_checksum(self, header_offset, length, recyclable):
        hs = K_RECYCLABLE_HEADER if recyclable else K_HEADER
        d = bytes(self.w.buf[header_offset + 6:header_offset + hs + length])
        struct.pack_into("<I", self.w.buf, header_offset, self.o.Mask(self.o.Value(d)))


def cases():
    """(name, build(log), mode, expected records, check(dropped, message))."""
    C = []

    def add(name, build, records, check=None, mode=kTolerate, recycle_only=None):
        C.append((name, build, mode, records, check, recycle_only))

    add("Empty", lambda L: None, lambda L: [])
    add("ReadWrite", lambda L: [L.write(m) for m in (b"foo", b"bar", b"", b"xxxx")],
        lambda L: [b"foo", b"bar", b"", b"xxxx"])
    add("ManyBlocks", lambda L: [L.write(number_string(i)) for i in range(100000)],
        lambda L: [number_string(i) for i in range(100000)])
    add("Fragmentation", lambda L: [L.write(m) for m in (b"small", big_string("medium", 50000),
                                                         big_string("large", 100000))],
        lambda L: [b"small", big_string("medium", 50000), big_string("large", 100000)])

    def marginal(L):
        n = K_BLOCK - 2 * L.hs
        L.write(big_string("foo", n))
        assert L.written() == K_BLOCK - L.hs
        L.write(b"")
        L.write(b"bar")
    add("MarginalTrailer", marginal,
        lambda L: [big_string("foo", K_BLOCK - 2 * L.hs), b"", b"bar"])

    def marginal2(L):
        n = K_BLOCK - 2 * L.hs
        L.write(big_string("foo", n))
        assert L.written() == K_BLOCK - L.hs
        L.write(b"bar")
    add("MarginalTrailer2", marginal2, lambda L: [big_string("foo", K_BLOCK - 2 * L.hs), b"bar"],
        lambda d, m: d == 0 and m == "")

    def short_trailer(L):
        n = K_BLOCK - 2 * L.hs + 4
        L.write(big_string("foo", n))
        assert L.written() == K_BLOCK - L.hs + 4
        L.write(b"")
        L.write(b"bar")
    add("ShortTrailer", short_trailer,
        lambda L: [big_string("foo", K_BLOCK - 2 * L.hs + 4), b"", b"bar"])

    def aligned_eof(L):
        n = K_BLOCK - 2 * L.hs + 4
        L.write(big_string("foo", n))
        assert L.written() == K_BLOCK - L.hs + 4
    add("AlignedEof", aligned_eof, lambda L: [big_string("foo", K_BLOCK - 2 * L.hs + 4)])

    def bad_record_type(L):  # :429-437
        L.write(b"foo")
        L.increment_byte(6, 100)
        L.fix_checksum(0, 3, False)
    add("BadRecordType", bad_record_type, lambda L: [],
        lambda d, m: d == 3 and "unknown record type" in m)

    def truncated_trailing(L):  # :439-460
        L.write(b"foo")
        L.shrink(4)
    add("TruncatedTrailingRecordIsIgnored", truncated_trailing, lambda L: [],
        lambda d, m: d == 0 and m == "")
    add("TruncatedTrailingRecordIsNotIgnored", truncated_trailing, lambda L: [],
        lambda d, m: d > 0 and "Corruption: truncated header" in m, mode=kAbsolute)

    def bad_length(L):  # :462-483
        L.write(big_string("bar", K_BLOCK - L.hs))
        L.write(b"foo")
        L.increment_byte(4, 1)
    add("BadLength", bad_length, lambda L: [b"foo"] if not L.recycle else [],
        lambda d, m: (d == K_BLOCK and "bad record length" in m), recycle_only=False)
    add("BadLength", bad_length, lambda L: [], lambda d, m: True, recycle_only=True)

    def bad_length_at_end(L):  # :485-511
        L.write(b"foo")
        L.shrink(1)
    add("BadLengthAtEndIsIgnored", bad_length_at_end, lambda L: [], lambda d, m: d == 0 and m == "")
    add("BadLengthAtEndIsNotIgnored", bad_length_at_end, lambda L: [],
        lambda d, m: d > 0 and "Corruption: truncated record body" in m, mode=kAbsolute)

    def checksum_mismatch(L):  # :513-525
        L.write(b"foooooo")
        L.increment_byte(0, 14)
    add("ChecksumMismatch", checksum_mismatch, lambda L: [],
        lambda d, m: d == 14 and "checksum mismatch" in m, recycle_only=False)
    add("ChecksumMismatch", checksum_mismatch, lambda L: [], lambda d, m: d == 0 and m == "",
        recycle_only=True)

    def unexpected(t_legacy, t_recycle, extra=()):
        def build(L):
            L.write(b"foo")
            for e in extra:
                L.write(e)
            L.set_byte(6, t_recycle if L.recycle else t_legacy)
            L.fix_checksum(0, 3, L.recycle)
        return build
    add("UnexpectedMiddleType", unexpected(kMiddleType, kRecyclableMiddleType), lambda L: [],
        lambda d, m: d == 3 and "missing start" in m)
    add("UnexpectedLastType", unexpected(kLastType, kRecyclableLastType), lambda L: [],
        lambda d, m: d == 3 and "missing start" in m)
    add("UnexpectedFullType", unexpected(kFirstType, kRecyclableFirstType, (b"bar",)), lambda L: [b"bar"],
        lambda d, m: d == 3 and "partial record without end" in m)
    add("UnexpectedFirstType", unexpected(kFirstType, kRecyclableFirstType, (big_string("bar", 100000),)),
        lambda L: [big_string("bar", 100000)], lambda d, m: d == 3 and "partial record without end" in m)

    def missing_last(L):  # :590-611
        L.write(big_string("bar", K_BLOCK))
        L.shrink(14)
    add("MissingLastIsIgnored", missing_last, lambda L: [], lambda d, m: d == 0 and m == "")
    add("MissingLastIsNotIgnored", missing_last, lambda L: [],
        lambda d, m: d > 0 and "Corruption: error reading trailing data" in m, mode=kAbsolute)

    def partial_last(L):  # :613-634
        L.write(big_string("bar", K_BLOCK))
        L.shrink(1)
    add("PartialLastIsIgnored", partial_last, lambda L: [], lambda d, m: d == 0 and m == "")
    add("PartialLastIsNotIgnored", partial_last, lambda L: [],
        lambda d, m: d > 0 and "Corruption: truncated record body" in m, mode=kAbsolute)

    def error_joins(L):  # :636-660
        L.write(big_string("foo", K_BLOCK))
        L.write(big_string("bar", K_BLOCK))
        L.write(b"correct")
        for off in range(K_BLOCK, 2 * K_BLOCK):
            L.set_byte(off, ord("x"))
    add("ErrorJoinsRecords", error_joins, lambda L: [b"correct"],
        lambda d, m: 2 * K_BLOCK <= d <= 2 * K_BLOCK + 100, recycle_only=False)
    add("ErrorJoinsRecords", error_joins, lambda L: [], None, recycle_only=True)

    def recycle(L):  # :717-742
        for m in (b"foo", b"bar", b"baz", b"bif", b"blitz"):
            L.write(m)
        while L.written() < K_BLOCK * 2:
            L.write(b"xxxxxxxxxxxxxxxx")
        # a new writer of the same log number overwrites the file from 0
        w2 = WalWriter(L.o, log_number=LOG, recycle=True)
        w2.add_record(b"foooo")
        w2.add_record(b"bar")
        L.w.buf[:len(w2.buf)] = w2.buf
        assert L.written() >= K_BLOCK * 2
    add("Recycle", recycle, lambda L: [b"foooo", b"bar"], None, recycle_only=True)
    return C


CASES = cases()
PARAMS = [(c, r) for c in CASES for r in (False, True) if c[5] is None or c[5] == r]
IDS = [f"{c[0]}-{'recycle' if r else 'legacy'}" for c, r in PARAMS]


def _records(plan, img):
    buf = bytearray(plan.records_bytes)
    for f in plan.frags[:plan.nfrags]:
        buf[f.dst_off:f.dst_off + f.length] = img[f.src_off:f.src_off + f.length]
    return [bytes(buf[int(o):int(o) + int(n)]) for o, n in zip(plan.rec_offsets, plan.rec_lengths)]


def _check(case, L, records, dropped, message):
    name, _, mode, want, chk, _ = case
    assert records == want(L), name
    if chk is not None:
        assert chk(dropped, message), (name, dropped, message)


@pytest.mark.parametrize("case,recycle", PARAMS, ids=IDS)
def test_log_reader_cases(oracle, case, recycle):
    import speedb_amd as S
    L = Log(oracle, recycle)
    case[1](L)
    img = bytes(L.w.buf)
    verified = np.array(wal_expected_blocks(img, LOG, oracle), dtype=np.int64).astype(np.int32) \
        if img else None
    plan = S.wal_read_records(img, LOG, case[2], verified)
    _check(case, L, _records(plan, img), plan.dropped_bytes, plan.message)


@pytest.mark.gpu
@pytest.mark.parametrize("case,recycle", PARAMS, ids=IDS)
def test_log_reader_cases_on_device(gpu, oracle, case, recycle):
    """The same cases with the CRC verdicts from mck_wal_verify_batch, the
    records reassembled by mck_wal_gather_batch and their XXH3
    record_checksum (ReadRecord's, db/log_reader.cc:107-158) from the
    device."""
    import speedb_amd as S
    L = Log(oracle, recycle)
    case[1](L)
    img = bytes(L.w.buf)
    r = S.WalRecover(img, LOG, case[2])
    recs = r.Records()
    _check(case, L, recs, r.dropped_bytes, r.message)
    assert [int(x) for x in r.record_checksums] == [oracle.XXH3(x) for x in recs]


def test_reader_reports_and_modes(oracle):
    """Report offsets/bytes and kSkipAnyCorruptedRecords: a corrupted
    record in the middle of the log is dropped with its block and reading
    continues in every mode but a recycled log's kTolerate."""
    import speedb_amd as S
    L = Log(oracle, False)
    msgs = [big_string(str(i), 20000) for i in range(8)]
    for m in msgs:
        L.write(m)
    # corrupt one payload byte of the record at the start of block 1
    first_in_block1 = next(off for off, _, _ in L.w.records if off >= K_BLOCK)
    L.increment_byte(first_in_block1 + K_HEADER + 5, 1)
    img = bytes(L.w.buf)
    ver = np.array(wal_expected_blocks(img, LOG, oracle), dtype=np.int64).astype(np.int32)
    for mode in (kTolerate, kAbsolute, kPIT, kSkipAny):
        plan = S.wal_read_records(img, LOG, mode, ver)
        recs = _records(plan, img)
        assert "checksum mismatch" in plan.message
        assert plan.reports[0][0] == first_in_block1
        assert plan.reports[0][1] == K_BLOCK - (first_in_block1 - K_BLOCK)  # rest of the block
        assert all(r in msgs for r in recs) and len(recs) < len(msgs)
        assert [int(x) for x in plan.rec_file_offsets] == sorted(int(x) for x in plan.rec_file_offsets)
    # results that do not describe this image are refused
    bad = ver.copy()
    bad[1, 1] = 0
    bad[1, 2] = 0
    with pytest.raises(Exception):
        S.wal_read_records(img, LOG, kTolerate, bad)


@pytest.mark.gpu
def test_wal_recover_on_side_stream(gpu, oracle):
    """WalRecover with stream= a busy non-default stream: the upload, the
    verify kernel, the host walk's readback and the XXH3 batch all order on
    that stream (the walk never reads verdicts not yet written)."""
    import speedb_amd as S
    torch = gpu
    L = Log(oracle, False)
    msgs = [big_string(str(i), 9000 + 37 * i) for i in range(40)]
    for m in msgs:
        L.write(m)
    img = bytes(L.w.buf)
    side = torch.cuda.Stream()
    big = torch.empty(1 << 28, dtype=torch.uint8, device="cuda")
    with torch.cuda.stream(side):
        for _ in range(8):
            big.fill_(3)  # the side stream is busy when WalRecover queues on it
    r = S.WalRecover(img, LOG, kTolerate, stream=side)
    assert r.Records() == msgs and r.dropped_bytes == 0
    assert [int(x) for x in r.record_checksums] == [oracle.XXH3(m) for m in msgs]


# ---------------------------------------------------------------------------
# FragmentBufferedReader (allow_retry_read = true, db/log_reader.cc:618-931):
# LogTest's cases that run for the retry reader (the ones log_test.cc skips
# with `if (allow_retry_read_) return;` are skipped here too), the ClearEof
# cases (ForceEOF = a shorter visible file, UnmarkEOF after it grew) and
# RetriableLogTest (:879-988, a record written in two parts).  ClearEofError
# / ClearEofError2 inject I/O errors into the file layer, which an in-memory
# image does not have: not restated.
# ---------------------------------------------------------------------------
RETRY_SKIPPED = {"TruncatedTrailingRecordIsNotIgnored", "BadLength", "BadLengthAtEndIsIgnored",
                 "BadLengthAtEndIsNotIgnored", "MissingLastIsNotIgnored", "PartialLastIsNotIgnored"}
RETRY_PARAMS = [(c, r) for c, r in PARAMS if c[0] not in RETRY_SKIPPED]
RETRY_IDS = [f"{c[0]}-{'recycle' if r else 'legacy'}" for c, r in RETRY_PARAMS]


def _tail_reader(oracle, verify):
    import speedb_amd as S
    if verify == "oracle":
        v = lambda img: wal_expected_blocks(img, LOG, oracle)  # noqa: E731
    else:
        v = verify
    return S.FragmentBufferedReader(LOG, verify=v)


def _read_all(r):
    out = []
    while True:
        rec = r.ReadRecord()
        if rec is None:
            return out
        out.append(rec)


def _retry_case(oracle, case, recycle, verify):
    L = Log(oracle, recycle)
    case[1](L)
    r = _tail_reader(oracle, verify)
    r.SetFile(bytes(L.w.buf))
    recs = _read_all(r)
    _check(case, L, recs, r.dropped_bytes, r.message)


@pytest.mark.parametrize("case,recycle", RETRY_PARAMS, ids=RETRY_IDS)
def test_fragment_buffered_reader_cases(oracle, case, recycle):
    _retry_case(oracle, case, recycle, "oracle")


def _clear_eof_single(oracle, recycle, verify):  # log_test.cc:649-664
    L = Log(oracle, recycle)
    L.write(b"foo")
    L.write(b"bar")
    r = _tail_reader(oracle, verify)
    r.SetFile(bytes(L.w.buf[:3 + L.hs + 2]))  # ForceEOF(3 + header_size + 2)
    assert r.ReadRecord() == b"foo"
    r.SetFile(bytes(L.w.buf))
    r.UnmarkEOF()
    assert r.ReadRecord() == b"bar"
    assert r.IsEOF()
    assert r.ReadRecord() is None
    L.write(b"xxx")
    r.SetFile(bytes(L.w.buf))
    r.UnmarkEOF()
    assert r.ReadRecord() == b"xxx"
    assert r.IsEOF()


def _clear_eof_multi(oracle, recycle, verify):  # log_test.cc:666-683
    L = Log(oracle, recycle)
    blocks = 5
    n = (K_BLOCK - L.hs) * blocks + 25
    L.write(big_string("foo", n))
    L.write(big_string("bar", n))
    r = _tail_reader(oracle, verify)
    r.SetFile(bytes(L.w.buf[:n + blocks * L.hs + L.hs + 3]))
    assert r.ReadRecord() == big_string("foo", n)
    assert r.IsEOF()
    r.SetFile(bytes(L.w.buf))
    r.UnmarkEOF()
    assert r.ReadRecord() == big_string("bar", n)
    assert r.IsEOF()
    L.write(big_string("xxx", n))
    r.SetFile(bytes(L.w.buf))
    r.UnmarkEOF()
    assert r.ReadRecord() == big_string("xxx", n)
    assert r.IsEOF()


def _tail_two_parts(oracle, recycle, verify, delta_of_hs, msg):
    """RetriableLogTest TailLog_PartialHeader (:879, delta = hs - 1),
    TailLog_FullHeader (:922, hs + 1), NonBlockingReadFullRecord (:965):
    the reader polls while the record is written in two parts."""
    L = Log(oracle, recycle)
    L.write(msg)
    img = bytes(L.w.buf)
    delta = delta_of_hs(L.hs)
    r = _tail_reader(oracle, verify)
    r.SetFile(img[:delta])
    assert r.ReadRecord() is None
    assert r.IsEOF()  # the FirstEOF sync point was reached
    r.SetFile(img)
    assert r.ReadRecord() == msg
    assert r.dropped_bytes == 0 and r.message == ""


def _tail_byte_by_byte(oracle, recycle, verify):
    """A log written a few bytes at a time, polled after every write: every
    record comes out once, whole, in order (the secondary-instance loop)."""
    import random
    L = Log(oracle, recycle)
    rnd = random.Random(9)
    msgs = [big_string(str(i), rnd.choice([0, 1, 5, 100, 3000, 40000])) for i in range(40)]
    for m in msgs:
        L.write(m)
    img = bytes(L.w.buf)
    r = _tail_reader(oracle, verify)
    got, pos = [], 0
    while pos < len(img):
        pos = min(len(img), pos + rnd.choice([1, 3, 7, 11, 500, 9000, 33000]))
        r.SetFile(img[:pos])
        got += _read_all(r)
    assert got == msgs and r.dropped_bytes == 0


def _tail_corrupt_then_append(oracle, recycle, verify):
    """A checksum failure in a partly written block, then more records
    appended to the same block: the failure drops only the buffer
    up to the file's end (db/log_reader.cc:889-891 buffer_.clear()), the
    reader reads on behind it (TryReadMore -> UnmarkEOF, :340-397, :785-823)
    and returns every appended record; the bad record is reported once
    (legacy) or ends the read silently (recyclable, :757-760)."""
    L = Log(oracle, recycle)
    L.write(b"foo")
    bar_hdr = L.written()
    L.write(b"bar")
    L.increment_byte(bar_hdr + L.hs, 1)  # a payload byte of "bar"
    r = _tail_reader(oracle, verify)
    r.SetFile(bytes(L.w.buf))
    assert r.ReadRecord() == b"foo"
    assert r.ReadRecord() is None
    _, first_dropped = r._reports()[1], r.dropped_bytes
    L.write(b"baz")
    L.write(big_string("qux", 1000))
    r.SetFile(bytes(L.w.buf))
    r.UnmarkEOF()
    assert _read_all(r) == [b"baz", big_string("qux", 1000)]
    reps, dropped = r._reports()
    if recycle:
        assert reps == [] and dropped == 0
    else:
        assert [(x[1], x[2]) for x in reps] == [(L.hs + 3, "checksum mismatch")]
        assert dropped == first_dropped == L.hs + 3
    assert r.OldRecordOffset() is None


def _tail_old_record(oracle, recycle, verify):
    """A recycled log whose tail still holds a record of the previous log
    instance: the reader stops there and says so (OldRecordOffset), however
    the file grows."""
    if not recycle:
        return
    L = Log(oracle, recycle)
    L.write(b"foo")
    stale = WalWriter(oracle, log_number=LOG - 1, recycle=True)
    stale.add_record(b"old!")
    at = L.written()
    L.w.buf += stale.buf
    r = _tail_reader(oracle, verify)
    r.SetFile(bytes(L.w.buf))
    assert r.ReadRecord() == b"foo"
    assert r.ReadRecord() is None
    assert r.OldRecordOffset() == at
    r.SetFile(bytes(L.w.buf) + b"\0" * 100)
    assert r.ReadRecord() is None and r.OldRecordOffset() == at


TAIL_CASES = {
    "CorruptThenAppend": _tail_corrupt_then_append,
    "OldRecordStall": _tail_old_record,
    "ClearEofSingleBlock": _clear_eof_single,
    "ClearEofMultiBlock": _clear_eof_multi,
    "TailLog_PartialHeader": lambda o, rc, v: _tail_two_parts(o, rc, v, lambda hs: hs - 1, b"foo"),
    "TailLog_FullHeader": lambda o, rc, v: _tail_two_parts(o, rc, v, lambda hs: hs + 1, b"foo"),
    "NonBlockingReadFullRecord": lambda o, rc, v: _tail_two_parts(o, rc, v, lambda hs: hs - 1, b"foo-bar"),
    "ByteByByte": _tail_byte_by_byte,
}


@pytest.mark.parametrize("recycle", [False, True])
@pytest.mark.parametrize("name", list(TAIL_CASES))
def test_fragment_buffered_reader_tailing(oracle, name, recycle):
    TAIL_CASES[name](oracle, recycle, "oracle")


def test_timestamp_size_record_offsets(oracle):
    """A user-defined timestamp size record (type 10) in the middle of a
    fragmented record: ReadRecord reports it interspersed and the record that
    then completes has LastRecordOffset = the timestamp record's offset
    (db/log_reader.cc:189-213); a zero size and a second record for the same
    column family are reported by UpdateRecordedTimestampSize (:594-616)."""
    import speedb_amd as S
    L = Log(oracle, False)
    L.write(b"head")
    L.w.emit(kFirstType, b"abc")
    ts_off = len(L.w.buf)
    L.w.emit(10, struct.pack("<IH", 1, 8))    # cf 1 -> 8-byte timestamps, inside the record
    L.w.emit(kLastType, b"def")
    L.w.emit(10, struct.pack("<IH", 2, 0))    # zero size
    L.w.emit(10, struct.pack("<IH", 1, 4))    # cf 1 again
    L.write(b"tail")
    img = bytes(L.w.buf)
    ver = np.array(wal_expected_blocks(img, LOG, oracle), dtype=np.int64).astype(np.int32)
    plan = S.wal_read_records(img, LOG, kTolerate, ver)
    assert _records(plan, img) == [b"head", b"def", b"tail"]
    assert int(plan.rec_file_offsets[1]) == ts_off
    assert [(rep[1], rep[2]) for rep in plan.reports] == [
        (3, "user-defined timestamp size record interspersed partial record"),
        (6, "User-defined timestamp size record contains zero timestamp size."),
        (6, "User-defined timestamp size record contains update to recorded column family.")]


@pytest.mark.gpu
@pytest.mark.parametrize("case,recycle", RETRY_PARAMS, ids=RETRY_IDS)
def test_fragment_buffered_reader_cases_on_device(gpu, oracle, case, recycle):
    """The same cases with the CRC verdicts from mck_wal_verify_batch."""
    _retry_case(oracle, case, recycle, "device")


@pytest.mark.gpu
@pytest.mark.parametrize("recycle", [False, True])
@pytest.mark.parametrize("name", list(TAIL_CASES))
def test_fragment_buffered_reader_tailing_on_device(gpu, oracle, name, recycle):
    """Tailing with the device verdicts: every SetFile re-verifies the
    blocks that grew (a partly written block verified again)."""
    TAIL_CASES[name](oracle, recycle, "device")


# ---------------------------------------------------------------------------
# WAL compression (db/log_writer.cc AddCompressionTypeRecord, db/log_reader.cc
# :167-188 ReadRecord's kSetCompressionType case, :529-571 the uncompressor
# fed by ReadPhysicalRecord).  The engine walks and CRC-verifies a compressed
# log like any other; its records come back as the compressed chunks plus the
# stream of every chunk the reference feeds its StreamingUncompress (the
# decompression itself is the caller's).  The chunks here are opaque bytes:
# no zstd in this image, and the walk never looks inside them.
# ---------------------------------------------------------------------------
kSetCompressionType, kZSTD = 9, 7


def _compressed_log(oracle, recycle, ctype=kZSTD):
    L = Log(oracle, recycle)
    L.w.emit(kSetCompressionType, struct.pack("<I", ctype))
    return L


def _stream_ok(plan, img):
    """Every stream entry that belongs to a returned record names that
    record's fragment, in order."""
    fr = plan.frags
    for off, n, k in plan.stream:
        if k >= 0:
            assert (fr[k].src_off, fr[k].length) == (off, n)
    kept = [k for _, _, k in plan.stream if k >= 0]
    assert kept == sorted(kept) == list(range(plan.nfrags))


@pytest.mark.parametrize("recycle", [False, True])
def test_compressed_wal_walk(oracle, recycle):
    """CompressionLogTest.ReadWrite / ManyBlocks / Fragmentation shapes
    (log_test.cc:1012-1130): the compression record first, then chunks."""
    import speedb_amd as S
    L = _compressed_log(oracle, recycle)
    chunks = [b"foo", b"bar", b"", b"xxxx", big_string("medium", 50000), big_string("large", 100000)]
    chunks += [number_string(i) for i in range(1000)]
    for c in chunks:
        L.write(c)
    img = bytes(L.w.buf)
    ver = np.array(wal_expected_blocks(img, LOG, oracle), dtype=np.int64).astype(np.int32)
    plan = S.wal_read_records(img, LOG, kTolerate, ver)
    assert plan.compression_type == kZSTD
    assert _records(plan, img) == chunks and plan.reports == []
    # every physical record after the compression record is one chunk of the stream
    assert [img[o:o + n] for o, n, _ in plan.stream] == [img[f.src_off:f.src_off + f.length]
                                                         for f in plan.frags[:plan.nfrags]]
    _stream_ok(plan, img)


def test_read_out_struct_size(oracle):
    """mck_wal_read_out carries its caller's struct_size: 0 is
    refused, and a caller built against the layout without the compression
    fields gets MCK_ENOTSUP for a compressed WAL, with nothing written past
    its struct; an uncompressed WAL reads the same with either size."""
    import ctypes
    from speedb_amd import checksum as C
    from speedb_amd._lib import lib
    L = _compressed_log(oracle, False)
    for c in (b"foo", b"bar" * 100):
        L.write(c)
    img = bytes(L.w.buf)

    class Guarded(ctypes.Structure):
        _fields_ = [("o", C.mck_wal_read_out), ("guard", ctypes.c_uint64 * 8)]

    g = Guarded()
    assert lib.mck_wal_read_records(img, len(img), LOG, kTolerate, None, ctypes.addressof(g.o)) == -1
    g.o.struct_size = 120  # MCK_WAL_READ_OUT_V1_SIZE
    # the v1 struct ends at compression_type: fill everything past it
    ctypes.memset(ctypes.addressof(g) + 120, 0xCD, ctypes.sizeof(g) - 120)
    rc = lib.mck_wal_read_records(img, len(img), LOG, kTolerate, None, ctypes.addressof(g.o))
    assert rc == -6 and "compression" in lib.mck_last_error().decode()  # MCK_ENOTSUP
    assert bytes((ctypes.c_uint8 * (ctypes.sizeof(g) - 120)).from_address(ctypes.addressof(g) + 120)) == \
        b"\xcd" * (ctypes.sizeof(g) - 120)
    w = WalWriter(oracle, LOG)
    for c in (b"foo", b"bar" * 100):
        w.add_record(c)
    plain = bytes(w.buf)
    for size in (120, ctypes.sizeof(C.mck_wal_read_out)):
        o = C.mck_wal_read_out()
        o.struct_size = size
        assert lib.mck_wal_read_records(plain, len(plain), LOG, kTolerate, None, ctypes.addressof(o)) == 0
        assert o.nrecords == 2


def test_compressed_wal_corruption_and_drops(oracle):
    """A chunk whose CRC fails is dropped BEFORE the uncompressor (not in the
    stream); a first fragment whose record never completes WAS fed (in the
    stream, belonging to no record)."""
    import speedb_amd as S
    L = _compressed_log(oracle, False)
    L.write(b"aaaa")
    bad_at = L.written()
    L.write(b"bbbbbbbb")
    L.increment_byte(bad_at + K_HEADER + 2, 1)  # payload byte of the 2nd record
    L.w.emit(kFirstType, b"orphan-first")       # a record that never ends...
    L.write(b"cccc")                            # ...interrupted by a full record
    img = bytes(L.w.buf)
    ver = np.array(wal_expected_blocks(img, LOG, oracle), dtype=np.int64).astype(np.int32)
    plan = S.wal_read_records(img, LOG, kTolerate, ver)
    assert plan.compression_type == kZSTD
    assert _records(plan, img) == [b"aaaa"]     # the CRC failure drops the rest of the block
    assert [r[2] for r in plan.reports] == ["checksum mismatch"]
    # the same after the block: the failed chunk is not fed, the orphan first is
    L2 = _compressed_log(oracle, False)
    L2.write(b"aaaa")
    L2.w.buf += b"\0" * (K_BLOCK - len(L2.w.buf))  # next block
    L2.w.block_offset = 0
    L2.w.emit(kFirstType, b"orphan-first")
    L2.write(b"cccc")
    img2 = bytes(L2.w.buf)
    ver2 = np.array(wal_expected_blocks(img2, LOG, oracle), dtype=np.int64).astype(np.int32)
    plan2 = S.wal_read_records(img2, LOG, kTolerate, ver2)
    assert _records(plan2, img2) == [b"aaaa", b"cccc"]
    assert [r[2] for r in plan2.reports] == ["partial record without end(1)"]
    chunks = [img2[o:o + n] for o, n, _ in plan2.stream]
    assert chunks[:2] == [b"aaaa", b""] or chunks[0] == b"aaaa"
    assert b"orphan-first" in chunks and [k for o, n, k in plan2.stream if img2[o:o + n] == b"orphan-first"] == [-1]
    _stream_ok(plan2, img2)


def test_compressed_recyclable_log_bad_crc_goes_on(oracle):
    """A recyclable compressed log starts with kSetCompressionType under the
    legacy 7-byte header, so ReadPhysicalRecord never sets recycled_
    (log_reader.cc:472-476: only a recyclable type at file offset 0 does) and
    a bad CRC under kTolerateCorruptedTailRecords does NOT end the log
    (:290-295): the rest of the block is dropped and reported, reading goes
    on.  (The same corruption in an uncompressed recyclable log ends it.)"""
    import speedb_amd as S
    L = _compressed_log(oracle, True)
    chunks = [big_string(str(i), 700 + 37 * i) for i in range(200)]
    for c in chunks:
        L.write(c)
    bad_at = L.w.records[-50][0]
    img = bytearray(L.w.buf)
    img[bad_at + K_RECYCLABLE_HEADER + 1] ^= 1
    img = bytes(img)
    ver = np.array(wal_expected_blocks(img, LOG, oracle), dtype=np.int64).astype(np.int32)
    plan = S.wal_read_records(img, LOG, kTolerate, ver)
    got = _records(plan, img)
    i = next(j for j, (a, b) in enumerate(zip(got, chunks)) if a != b)
    k = chunks.index(got[i])
    assert k > i and got[:i] == chunks[:i] and got[i:] == chunks[k:]
    # the drop, then the dropped record's later fragments in the next block
    assert [r[2] for r in plan.reports][0] == "checksum mismatch"
    assert all(r[2] == "checksum mismatch" or r[2].startswith("missing start") for r in plan.reports)


def test_compression_record_reports(oracle):
    """ReadRecord's kSetCompressionType checks (log_reader.cc:167-188)."""
    import speedb_amd as S
    # a second compression record after a record was read: both reports
    L = _compressed_log(oracle, False)
    L.write(b"one")
    L.w.emit(kSetCompressionType, struct.pack("<I", kZSTD))
    L.write(b"two")
    img = bytes(L.w.buf)
    plan = S.wal_read_records(img, LOG, kTolerate, None)
    assert _records(plan, img) == [b"one", b"two"]
    assert [(r[1], r[2]) for r in plan.reports] == [(4, "read multiple SetCompressionType records"),
                                                    (4, "SetCompressionType not the first record")]
    # an undecodable type (not streaming-capable) or a short record: reported,
    # the log is read uncompressed
    for payload in (struct.pack("<I", 3), b"\x07\x00"):
        L = Log(oracle, False)
        L.w.emit(kSetCompressionType, payload)
        L.write(b"plain")
        img = bytes(L.w.buf)
        plan = S.wal_read_records(img, LOG, kTolerate, None)
        assert plan.compression_type == 0 and plan.stream == []
        assert _records(plan, img) == [b"plain"]
        assert [(r[1], r[2]) for r in plan.reports] == [(len(payload), "could not decode SetCompressionType record")]
    # kNoCompression: accepted, nothing to uncompress
    L = _compressed_log(oracle, False, ctype=0)
    L.write(b"plain")
    img = bytes(L.w.buf)
    plan = S.wal_read_records(img, LOG, kTolerate, None)
    assert plan.compression_type == 0 and plan.reports == [] and _records(plan, img) == [b"plain"]


@pytest.mark.gpu
def test_compressed_wal_recover_on_device(gpu, oracle):
    """WalRecover on a compressed log: the device verifies every physical
    record's CRC (the compressed chunks are what the CRCs cover), the host
    walk returns the chunks; no XXH3 record checksum (it is over the
    decompressed bytes)."""
    import speedb_amd as S
    L = _compressed_log(oracle, True)
    chunks = [big_string(str(i), 700 + 37 * i) for i in range(200)]
    for c in chunks:
        L.write(c)
    bad_at = L.w.records[-50][0]
    img = bytearray(L.w.buf)
    img[bad_at + K_RECYCLABLE_HEADER + 1] ^= 1
    r = S.WalRecover(bytes(img), LOG, kTolerate)
    assert r.compression_type == kZSTD and r.record_checksums is None
    got = r.Records()
    # the log's first record is kSetCompressionType, written with the legacy
    # header (log_writer.cc EmitPhysicalRecord), so the reader never sets
    # recycled_ (log_reader.cc:472-476, only a recyclable type at offset 0
    # does): the bad CRC drops the rest of its block, is reported, and the
    # walk goes on -- unlike an uncompressed recyclable log, where it ends
    i = next(j for j, (a, b) in enumerate(zip(got, chunks)) if a != b)
    k = chunks.index(got[i])
    assert k > i and got[:i] == chunks[:i] and got[i:] == chunks[k:]
    assert any("checksum mismatch" in rep[2] for rep in r.reports), r.reports
    want = wal_expected_blocks(bytes(img), LOG, oracle)
    assert [tuple(int(x) for x in b) for b in r.blocks.cpu().numpy()] == [tuple(b) for b in want]

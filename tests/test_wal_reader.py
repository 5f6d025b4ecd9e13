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
record_checksum.  FragmentBufferedReader (allow_retry_read) and WAL
compression are not restated; cases that need them are skipped, as in the
reference."""
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

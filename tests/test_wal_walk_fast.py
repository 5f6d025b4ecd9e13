"""mck_wal_recover's plan walk from the block walk's list (wal_walk_fast,
round 6) against the reader's walk over the image (wal_walk, the
db/log_reader.cc restatement), host only: on clean logs the list walk runs
and every output equals the reader's (fragments, records, file offsets,
end offset, no reports); on logs with anything the list does not describe
(a corrupt length, a zero record, an old recyclable record, a truncated
tail, a middle / last fragment without its first, unknown types) it
declines and the reader's walk stays the plan.  Through the test hook
mck_test_wal_walk_fast (no GPU)."""
import random

import pytest

from formats import K_BLOCK, WalWriter

LOG = 77


def _walk(lib, img: bytes, log=LOG) -> int:
    return lib.mck_test_wal_walk_fast(img, len(img), log)


def _log(oracle, lens, recycle=False, seed=1):
    rnd = random.Random(seed)
    w = WalWriter(oracle, log_number=LOG, recycle=recycle)
    for n in lens:
        w.add_record(bytes(rnd.randrange(256) for _ in range(min(n, 64))) * (n // 64) +
                     bytes(n % 64) if n else b"")
    return w


@pytest.fixture(scope="module")
def lib():
    from speedb_amd._lib import lib
    return lib


@pytest.mark.parametrize("recycle", [False, True])
def test_fast_walk_equals_reader_on_clean_logs(lib, oracle, recycle):
    rnd = random.Random(5 + recycle)
    edge = [0, 1, 6, 7, 100, K_BLOCK - 7, K_BLOCK - 11, K_BLOCK - 14, K_BLOCK, 3 * K_BLOCK + 5, 70000]
    for trial in range(12):
        lens = edge + [rnd.randrange(0, 5000) for _ in range(rnd.randrange(50, 400))]
        rnd.shuffle(lens)
        w = _log(oracle, lens, recycle, seed=trial)
        assert _walk(lib, bytes(w.buf)) == 1, trial
    # an empty log, one record, a log ending exactly at a block boundary
    assert _walk(lib, b"") == 1
    assert _walk(lib, bytes(_log(oracle, [10], recycle).buf)) == 1
    w = _log(oracle, [K_BLOCK - (11 if recycle else 7)], recycle)
    assert len(w.buf) == K_BLOCK and _walk(lib, bytes(w.buf)) == 1


def test_fast_walk_declines_what_the_list_does_not_describe(lib, oracle):
    w = _log(oracle, [300, 5000, 40000, 200, 90, 33000, 12], seed=3)
    img = bytearray(w.buf)
    recs = w.records  # (header offset, type, payload length)
    cases = []
    b = bytearray(img)  # a length past the block
    b[recs[1][0] + 4:recs[1][0] + 6] = (0xFFFF).to_bytes(2, "little")
    cases.append(b)
    b = bytearray(img)  # a zero record (type 0, length 0) in the middle of a block
    b[recs[4][0]:recs[4][0] + 7] = bytes(7)
    cases.append(b)
    b = bytearray(img)  # an unknown type
    b[recs[0][0] + 6] = 44
    cases.append(b)
    b = bytearray(img)  # a first fragment retyped as full: its middle / last come without a first
    first = next(r for r in recs if r[1] == 2)
    b[first[0] + 6] = 1
    cases.append(b)
    b = bytearray(img)  # a full record retyped as first: the next full comes inside a fragment
    full = next(r for r in recs if r[1] == 1)
    b[full[0] + 6] = 2
    cases.append(b)
    cases.append(img[:-3])  # a truncated tail
    for k, c in enumerate(cases):
        assert _walk(lib, bytes(c)) in (0, 1), k  # never a different walk
        assert _walk(lib, bytes(c)) == 0, k
    # a recyclable log read as another log's: old records
    wr = _log(oracle, [100, 200], recycle=True)
    assert _walk(lib, bytes(wr.buf), log=LOG + 1) == 0
    # timestamp-size and compression records decline (types 9 / 10)
    for t in (9, 10):
        b = bytearray(img)
        b[recs[0][0] + 6] = t
        assert _walk(lib, bytes(b)) == 0


def test_fast_walk_random_corruptions_never_differ(lib, oracle):
    """Byte flips anywhere in the headers: the list walk either declines or
    equals the reader's walk (never a third answer)."""
    rnd = random.Random(9)
    w = _log(oracle, [rnd.randrange(0, 9000) for _ in range(150)], seed=4)
    img = bytes(w.buf)
    heads = [r[0] for r in w.records]
    seen = set()
    for k in range(300):
        b = bytearray(img)
        h = rnd.choice(heads)
        p = h + rnd.randrange(0, 7)
        b[p] = rnd.randrange(256)
        r = _walk(lib, bytes(b))
        assert r in (0, 1), k
        seen.add(r)
    assert seen == {0, 1}

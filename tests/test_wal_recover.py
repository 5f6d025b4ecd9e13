"""WAL recovery in one device pass (mck_wal_recover_batch / mck_wal_recover,
row a11): every physical record's CRC32C (db/log_reader.cc:512-525) and the
XXH3_64bits record_checksum of every logical record ReadRecord returns
(:107-110 for one fragment, hashed in place by the same kernel; :128-158 for
fragmented records, gathered and hashed on the same stream) -- what
DBImpl::RecoverLogFiles asks for (db/db_impl/db_impl_open.cc:1217-1221).

Checked against the CPU oracle (util/xxhash.cc's XXH3_64bits restated,
pinned by the reference's own vectors) and against mck_wal_verify_batch's
per-block results for the same images (the CRC half must not change).  The
reader's own semantics (log_test.cc's cases) run through mck_wal_recover in
test_wal_reader.py::test_log_reader_cases_on_device."""
import numpy as np
import pytest

from formats import K_BLOCK, WalWriter

LOG = 77
kTolerate, kAbsolute, kPIT, kSkipAny = 0, 1, 2, 3


def _payload(rng, n):
    return rng.integers(0, 256, size=n, dtype=np.uint8).tobytes()


def _full_slots(w: WalWriter):
    """{(block, k): (file offset of header, payload length)} of every
    full-type physical record, k = its index among the block's full records."""
    out, cnt = {}, {}
    for off, t, n in w.records:
        if t in (1, 5):
            b = off // K_BLOCK
            k = cnt.get(b, 0)
            cnt[b] = k + 1
            out[(b, k)] = (off, n)
    return out


# payload lengths around the XXH3 length classes (16, 128, 240), the 1 KiB
# segment / 64-byte stripe grid and the wave unit (4 segments), and the
# largest one-block record (32761 / 32757 bytes)
EDGE_LENS = [0, 1, 3, 4, 8, 9, 16, 17, 128, 129, 239, 240, 241, 255, 256, 257, 1023, 1024, 1025, 1087, 1088,
             1089, 2047, 2048, 3071, 3072, 4095, 4096, 4097, 4160, 5120, 8191, 8192, 8193, 16383, 16384,
             16385, 20000, 32761]


def _image(oracle, recycle, lens, seed):
    rng = np.random.default_rng(seed)
    w = WalWriter(oracle, log_number=LOG, recycle=recycle)
    recs = []
    for n in lens:
        p = _payload(rng, n)
        w.add_record(p)
        recs.append(p)
    return w, recs


def _plan(S, torch, img):
    plan = S.wal_plan_records(img, LOG)
    return plan, torch.from_numpy(plan.view(np.int32)).cuda()


def test_plan_records_lists_every_physical_record(oracle):
    """mck_wal_plan_records (host) = the writer's physical records: payload
    offset, type, length, stored CRC, the hash flag on full types."""
    import speedb_amd as S
    for recycle in (False, True):
        w, _ = _image(oracle, recycle, EDGE_LENS, 2)
        img = bytes(w.buf)
        plan = S.wal_plan_records(img, LOG)
        hs = 11 if recycle else 7
        assert len(plan) == len(w.records)
        for (off, t, n), d in zip(w.records, plan):
            assert int(d[0]) | ((int(d[1]) & 0xFFFF) << 32) == off + hs
            assert (int(d[1]) >> 16) & 0xFF == t and int(d[2]) == n
            assert int(d[3]) == int.from_bytes(img[off:off + 4], "little")
            assert bool(int(d[1]) & (1 << 24)) == (t in (1, 5))


@pytest.mark.gpu
@pytest.mark.parametrize("recycle", [False, True])
def test_recover_batch_equals_oracle(gpu, oracle, recycle):
    """Every physical record's CRC verdict holds and every full record's hash
    equals the oracle's XXH3 of its payload, for the edge lengths (XXH3's
    length classes, the 1 KiB segment / 64-B stripe grid, the last round's
    lane boundaries) at every payload alignment the headers produce."""
    import speedb_amd as S
    torch = gpu
    rng = np.random.default_rng(5)
    lens = EDGE_LENS * 3 + [int(x) for x in rng.integers(0, 40000, size=60)]
    rng.shuffle(lens)
    w, _ = _image(oracle, recycle, lens, 11)
    img = bytes(w.buf)
    # exactly 16 bytes of slack past the image (mck.h: readable 16 B past nbytes)
    d = torch.frombuffer(bytearray(img + bytes(16)), dtype=torch.uint8).cuda()
    plan, dp = _plan(S, torch, img)
    ok, h = S.wal_recover_batch(d, dp, LOG)
    assert (ok.cpu().numpy() == 1).all()
    hv = h.cpu().numpy().view(np.uint64)
    hs = 11 if recycle else 7
    for k, (off, t, n) in enumerate(w.records):
        if t in (1, 5):
            assert int(hv[k]) == oracle.XXH3(img[off + hs:off + hs + n]), (k, n, (off + hs) & 3)


@pytest.mark.gpu
def test_recover_batch_every_alignment_and_length(gpu, oracle):
    """Payloads of 0..1100 B and around 2-4 KiB at all four dword
    alignments, packed back to back in one image (legacy and recyclable
    headers mixed): verdicts all hold and every hash matches."""
    import speedb_amd as S
    torch = gpu
    rng = np.random.default_rng(77)
    lens = list(range(0, 1100, 7)) + [int(x) for x in rng.integers(1900, 4300, size=80)]
    rng.shuffle(lens)
    w = WalWriter(oracle, log_number=LOG, recycle=False)
    w2 = WalWriter(oracle, log_number=LOG, recycle=True)
    for n in lens:
        p = _payload(rng, n)
        (w if n % 2 else w2).add_record(p)
    for ww in (w, w2):
        img = bytes(ww.buf)
        d = torch.frombuffer(bytearray(img + bytes(16)), dtype=torch.uint8).cuda()
        plan, dp = _plan(S, torch, img)
        ok, h = S.wal_recover_batch(d, dp, LOG)
        assert (ok.cpu().numpy() == 1).all()
        hv = h.cpu().numpy().view(np.uint64)
        hs = 11 if ww.recycle else 7
        for k, (off, t, n) in enumerate(ww.records):
            if t in (1, 5):
                assert int(hv[k]) == oracle.XXH3(img[off + hs:off + hs + n]), (k, n)


@pytest.mark.gpu
@pytest.mark.parametrize("recycle", [False, True])
def test_recover_corrupt_records(gpu, oracle, recycle):
    """A flipped payload byte in a full record stops its block there (as
    ReadPhysicalRecord's kBadRecordChecksum drops the rest of the block);
    the records before it in the block keep their hashes; mck_wal_recover's
    walk then matches mck_wal_read_records over the same verdicts, with a
    checksum for every record it returns."""
    import speedb_amd as S
    torch = gpu
    rng = np.random.default_rng(21)
    lens = [int(x) for x in rng.integers(100, 6000, size=300)]
    w, _ = _image(oracle, recycle, lens, 8)
    img = bytearray(w.buf)
    hs = 11 if recycle else 7
    fulls = [(o, n) for o, t, n in w.records if t in (1, 5) and n > 20]
    for o, n in fulls[5::37]:
        img[o + hs + n // 2] ^= 0x10
    img = bytes(img)
    d = torch.frombuffer(bytearray(img + bytes(64)), dtype=torch.uint8).cuda()
    ver = S.wal_verify_batch(d, len(img), LOG).cpu().numpy()
    assert (ver[:, 1] == 1).any()
    plan, dp = _plan(S, torch, img)
    ok, _ = S.wal_recover_batch(d, dp, LOG)
    bad = {o + hs + n // 2 for o, n in fulls[5::37]}
    want_ok = [0 if any(p <= x < p + n for x in bad) else 1
               for p, n in ((int(r[0]) | ((int(r[1]) & 0xFFFF) << 32), int(r[2])) for r in plan)]
    assert ok.cpu().numpy().tolist() == want_ok
    for mode in (kTolerate, kAbsolute, kPIT, kSkipAny):
        r = S.WalRecover(img, LOG, mode)
        plan = S.wal_read_records(img, LOG, mode, ver)
        assert r.message == plan.message and r.dropped_bytes == plan.dropped_bytes
        recs = r.Records()
        assert len(recs) == len(plan.rec_lengths)
        assert [int(x) for x in r.record_checksums] == [oracle.XXH3(x) for x in recs]
        assert r.info.host_walks == 2
        # the per-block verdicts derived from the per-record ones are the
        # device walk's (mck_wal_verify_batch)
        assert (r.blocks.numpy() == ver).all()


@pytest.mark.gpu
@pytest.mark.parametrize("recycle", [False, True])
def test_wal_recover_mixed_records_at_scale(gpu, oracle, recycle):
    """A group-commit-shaped log written by the device writer (records of
    100 B - 4 KiB, the realistic mix the bench times): every record and
    every record_checksum bit-exact, the one-fragment records hashed in the
    recover pass, the block-straddling ones gathered."""
    import speedb_amd as S
    torch = gpu
    rng = np.random.default_rng(31)
    n = 40000
    lens = rng.integers(100, 4097, size=n).astype(np.int64)
    offs = np.zeros(n, np.int64)
    offs[1:] = np.cumsum(lens)[:-1]
    src = torch.randint(0, 256, (int(lens.sum()) + 64,), dtype=torch.uint8, device="cuda")
    log = S.WalBatchWriter(LOG, recycle_log_files=recycle).AddRecords(src, offs, lens)
    img = bytes(log.cpu().numpy().tobytes())
    dev = torch.zeros(len(img) + 64, dtype=torch.uint8, device="cuda")
    dev[:len(img)] = log
    r = S.WalRecover(img, LOG, kTolerate, wal_dev=dev)
    host_src = src.cpu().numpy().tobytes()
    want = [host_src[o:o + k] for o, k in zip(offs, lens)]
    got = r.Records()
    assert got == want and r.dropped_bytes == 0
    assert [int(x) for x in r.record_checksums] == [oracle.XXH3(x) for x in want]
    assert r.info.in_place + r.info.gathered == n and r.info.gathered > 0 and r.info.in_place > 0
    assert r.info.host_walks == 1


@pytest.mark.gpu
def test_recover_configs3_shape(gpu, oracle):
    """configs[3]'s layout (one kFullType 32761-byte record per 32 KiB
    block, payloads at offset 7 of their block), more records than the grid
    has rows: every verdict holds, every hash equals the oracle's."""
    import speedb_amd as S
    from speedb_amd import workloads as W
    torch = gpu
    im = W.WalImage(6000, "cuda", seed=4, log_number=LOG)
    host = im.data[:im.nbytes].cpu().numpy()
    plan, dp = _plan(S, torch, host.tobytes())
    assert len(plan) == im.nblocks
    ok, h = S.wal_recover_batch(im.data, dp, LOG)
    assert (ok.cpu().numpy() == 1).all()
    hv = h.cpu().numpy().view(np.uint64)
    blocks = host.reshape(-1, K_BLOCK)
    for b in range(im.nblocks):
        assert int(hv[b]) == oracle.XXH3(blocks[b, 7:].tobytes()), b

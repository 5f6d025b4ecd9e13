"""Device WAL writer: the host plan fragments records
exactly as log::Writer::AddRecord does (compared with the test-side Python
restatement of db/log_writer.cc, tests/formats.py WalWriter), and the device
writes the same bytes -- legacy and recyclable headers, records spanning
blocks, empty records, block-trailer padding, an initial block offset."""
import random

import numpy as np
import pytest

from formats import WalWriter


def _records(seed, n, big=False):
    rnd = random.Random(seed)
    sizes = [0, 1, 7, 11, 32761, 32762, 32768, 70000] + [rnd.choice(
        [rnd.randrange(0, 100), rnd.randrange(0, 5000), rnd.randrange(30000, 100000 if big else 40000)])
        for _ in range(n)]
    rnd.shuffle(sizes)
    return [bytes(rnd.getrandbits(8) for _ in range(s)) for s in sizes]


@pytest.mark.parametrize("recycle", [False, True])
def test_wal_plan_matches_writer(oracle, recycle):
    import speedb_amd as S
    recs = _records(1, 60)
    w = WalWriter(oracle, log_number=123, recycle=recycle)
    # start mid-block like a log that already holds data
    pre = bytes(32768 - 9)
    w.add_record(pre[:32768 - 9 - (11 if recycle else 7)])
    start = len(w.buf)
    for r in recs:
        w.add_record(r)
    offs = np.cumsum([0] + [len(r) for r in recs[:-1]])
    frags, n, nbytes, nbo = S.wal_plan(offs, [len(r) for r in recs], start % 32768, recycle)
    assert nbytes == len(w.buf) - start
    assert nbo == w.block_offset
    got = [(f.dst_off + start, f.type, f.length) for f in frags[:n]]
    assert got == [r for r in w.records if r[0] >= start]


@pytest.mark.gpu
@pytest.mark.parametrize("recycle", [False, True])
def test_wal_write_batch_bit_exact(gpu, oracle, recycle):
    import torch

    import speedb_amd as S
    recs = _records(2, 300, big=True)
    w = WalWriter(oracle, log_number=77, recycle=recycle)
    w.add_record(b"x" * 1000)  # the log already holds one record
    start = len(w.buf)
    for r in recs:
        w.add_record(r)
    src = b"".join(recs)
    offs = np.cumsum([0] + [len(r) for r in recs[:-1]])
    dev = torch.frombuffer(bytearray(src + bytes(64)), dtype=torch.uint8).to("cuda")
    wr = S.WalBatchWriter(log_number=77, recycle_log_files=recycle, block_offset=start)
    out = wr.AddRecords(dev, offs, [len(r) for r in recs])
    got, want = bytes(out.cpu().numpy().tobytes()), bytes(w.buf[start:])
    if got != want:
        i = next(k for k in range(min(len(got), len(want))) if got[k] != want[k])
        fr = [r for r in w.records if r[0] <= i + start][-1]
        raise AssertionError(f"first difference at stream offset {i + start}: fragment {fr}")
    assert len(got) == len(want)
    assert wr.block_offset == w.block_offset
    # the device reader accepts every record of the full image
    full = torch.frombuffer(bytearray(bytes(w.buf) + bytes(64)), dtype=torch.uint8).to("cuda")
    res = S.wal_verify_batch(full, len(w.buf), 77).cpu().numpy()
    assert (res[:, 1] == 0).all()


@pytest.mark.gpu
@pytest.mark.parametrize("recycle", [False, True])
def test_wal_write_batch_large_group_commit(gpu, oracle, recycle):
    """A group commit of 24K records of 0..700 B with block-spanning ones
    (more fragments than one launch's descriptor cache on some GPUs): the
    stream is log::Writer's, byte for byte."""
    import torch

    import speedb_amd as S
    rng = np.random.default_rng(5)
    lens = rng.integers(0, 700, size=24000)
    lens[rng.integers(0, len(lens), size=40)] = rng.integers(30000, 70000, size=40)  # block-spanning ones
    src = rng.integers(0, 256, size=int(lens.sum()), dtype=np.uint8).tobytes()
    offs = np.concatenate([[0], np.cumsum(lens[:-1])])
    w = WalWriter(oracle, log_number=91, recycle=recycle)
    w.add_record(b"y" * 333)
    start = len(w.buf)
    for o, n in zip(offs, lens):
        w.add_record(src[o:o + n])
    dev = torch.frombuffer(bytearray(src + bytes(64)), dtype=torch.uint8).to("cuda")
    wr = S.WalBatchWriter(log_number=91, recycle_log_files=recycle, block_offset=start)
    out = wr.AddRecords(dev, offs, [int(n) for n in lens])
    got = out.cpu().numpy().tobytes()
    want = bytes(w.buf[start:])
    assert len(got) == len(want)
    if got != want:
        i = next(k for k in range(len(got)) if got[k] != want[k])
        raise AssertionError(f"first difference at stream offset {i + start}")


@pytest.mark.gpu
@pytest.mark.parametrize("recycle", [False, True])
def test_wal_write_batch_small_records_every_alignment(gpu, oracle, recycle):
    """Records of 0..80 bytes (a payload inside one output piece, head and
    tail bytes without a full piece, every output and source alignment) and
    a block-straddling tail: the one-pass writer's byte paths."""
    import torch

    import speedb_amd as S
    rng = np.random.default_rng(11)
    lens = np.concatenate([np.arange(0, 81), rng.integers(0, 300, size=3000), [32761, 5, 40000, 0, 17]])
    src = rng.integers(0, 256, size=int(lens.sum()) + 5, dtype=np.uint8).tobytes()
    offs = np.concatenate([[0], np.cumsum(lens[:-1])]) + 5  # source not 16-aligned either
    for start_pad in (0, 3, 11):
        w = WalWriter(oracle, log_number=0xABCD, recycle=recycle)
        if start_pad:
            w.add_record(b"z" * start_pad)
        start = len(w.buf)
        for o, n in zip(offs, lens):
            w.add_record(src[o:o + n])
        dev = torch.frombuffer(bytearray(src + bytes(64)), dtype=torch.uint8).to("cuda")
        wr = S.WalBatchWriter(log_number=0xABCD, recycle_log_files=recycle, block_offset=start)
        got = wr.AddRecords(dev, offs, [int(n) for n in lens]).cpu().numpy().tobytes()
        want = bytes(w.buf[start:])
        assert len(got) == len(want)
        if got != want:
            i = next(k for k in range(len(got)) if got[k] != want[k])
            raise AssertionError(f"start_pad {start_pad}: first difference at stream offset {i + start}")


@pytest.mark.gpu
@pytest.mark.parametrize("recycle", [False, True])
def test_wal_write_batch_round_boundaries(gpu, oracle, recycle):
    """Fragments whose cover sits at the one-pass writer's 1280-byte round
    boundaries (one round / two rounds / three), at every source offset mod
    16 and several output offsets: the piece that straddles two rounds is
    stored from the previous round's carried piece (k_wal_write_il), the
    CRC state crosses rounds through the 244-byte map."""
    import torch

    import speedb_amd as S
    rng = np.random.default_rng(23)
    base = [1200, 1249, 1250, 1264, 1265, 1266, 1279, 1280, 1281, 1296, 2500, 2529, 2545, 2560, 2561, 3830, 3840]
    lens = np.array([n + d for n in base for d in range(0, 16)] * 2, dtype=np.int64)
    rng.shuffle(lens)
    src = rng.integers(0, 256, size=int(lens.sum()) + 16, dtype=np.uint8).tobytes()
    for src_pad, start_pad in ((0, 0), (7, 5), (13, 9)):
        offs = np.concatenate([[0], np.cumsum(lens[:-1])]) + src_pad
        w = WalWriter(oracle, log_number=0x5151, recycle=recycle)
        if start_pad:
            w.add_record(b"q" * start_pad)
        start = len(w.buf)
        for o, n in zip(offs, lens):
            w.add_record(src[o:o + n])
        dev = torch.frombuffer(bytearray(src + bytes(64)), dtype=torch.uint8).to("cuda")
        wr = S.WalBatchWriter(log_number=0x5151, recycle_log_files=recycle, block_offset=start)
        got = wr.AddRecords(dev, offs, [int(n) for n in lens]).cpu().numpy().tobytes()
        want = bytes(w.buf[start:])
        assert len(got) == len(want)
        if got != want:
            i = next(k for k in range(len(got)) if got[k] != want[k])
            raise AssertionError(f"pads {src_pad}/{start_pad}: first difference at stream offset {i + start}")


@pytest.mark.gpu
def test_wal_write_batch_rejects_misaligned_out(gpu):
    import torch

    import speedb_amd as S
    from speedb_amd import _lib
    src = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    frags, nf, nbytes, _ = S.wal_plan([0], [100])
    d_frags = torch.frombuffer(bytearray(bytes(frags)), dtype=torch.uint8).to("cuda")
    crc = torch.zeros(4, dtype=torch.int32, device="cuda")
    out = torch.zeros(nbytes + 64, dtype=torch.uint8, device="cuda")
    rc = _lib.lib.mck_wal_write_batch(src.data_ptr(), d_frags.data_ptr(), nf, 0, crc.data_ptr(),
                                      out.data_ptr() + 1, None)
    assert rc == -1 and b"16-byte" in _lib.lib.mck_last_error()
    rc = _lib.lib.mck_wal_gather_batch(src.data_ptr(), d_frags.data_ptr(), nf, out.data_ptr() + 4, None)
    assert rc == -1
    assert _lib.lib.mck_wal_write_batch(src.data_ptr(), d_frags.data_ptr(), nf, 0, crc.data_ptr(),
                                        out.data_ptr(), None) == 0


@pytest.mark.parametrize("recycle", [False, True])
def test_wal_list_records_reassembly_plan(oracle, recycle):
    """log::Reader::ReadRecord's reassembly on the host: the logical records
    the writer produced, in order, with their fragments."""
    import speedb_amd as S
    recs = _records(3, 80)
    w = WalWriter(oracle, log_number=9, recycle=recycle)
    for r in recs:
        w.add_record(r)
    frags, nf, offs, lens, nbytes = S.wal_list_records(bytes(w.buf), 9)
    assert list(lens) == [len(r) for r in recs]
    assert nbytes == sum(len(r) for r in recs)
    assert nf == len(w.records)
    img = bytes(w.buf)
    buf = bytearray(nbytes)
    for f in frags[:nf]:
        buf[f.dst_off:f.dst_off + f.length] = img[f.src_off:f.src_off + f.length]
    for r, o, n in zip(recs, offs, lens):
        assert bytes(buf[o:o + n]) == r
    if recycle:  # a recycled log's records of another log number end the walk
        _, _, offs2, _, _ = S.wal_list_records(img, 10)
        assert len(offs2) == 0


def test_wal_list_records_drops_partial(oracle):
    """A record whose Last fragment is missing (the WAL ends mid-record) is
    dropped; a bad length drops the rest of its block."""
    import speedb_amd as S
    recs = [b"a" * 100, b"b" * 70000, b"c" * 50]
    w = WalWriter(oracle, log_number=1)
    for r in recs:
        w.add_record(r)
    img = bytes(w.buf)
    # cut inside the second record's Middle fragment: only record 0 survives
    cut = w.records[2][0] + 100
    _, _, offs, lens, _ = S.wal_list_records(img[:cut], 1)
    assert list(lens) == [100]


@pytest.mark.gpu
@pytest.mark.parametrize("recycle", [False, True])
def test_wal_read_records_xxh3(gpu, oracle, recycle):
    """Recovery on the device: reassembled records bit-exact, their
    XXH3_64bits (record_checksum) equal to the oracle's, every block's CRCs
    verified."""
    import speedb_amd as S
    recs = _records(4, 200, big=True)
    w = WalWriter(oracle, log_number=5, recycle=recycle)
    for r in recs:
        w.add_record(r)
    out, offs, lens, x3, blocks = S.WalReadRecords(bytes(w.buf), 5)
    host = bytes(out.cpu().numpy().tobytes())
    for r, o, n, h in zip(recs, offs, lens, x3):
        assert host[o:o + n] == r
        assert int(h) == oracle.XXH3(r)
    assert (blocks.cpu().numpy()[:, 1] == 0).all()


@pytest.mark.gpu
def test_wal_writer_stays_inside_its_buffers(gpu, oracle):
    """The one-pass writer never stores outside [out, out + nbytes) nor into
    the CRC scratch beyond its nfrags words: the output and scratch sit
    inside larger tensors whose 4 KiB guard regions (a canary pattern) must
    survive.  The first record starts at stream offset 0 (its first round's
    window begins up to 1280 bytes before the payload) and the last ends at
    the buffer's end (the review of the round-2 timing variant
    that faulted -- every piece, byte, header and CRC store of k_wal_write_il
    is guarded to the fragment's own bytes)."""
    import ctypes

    import torch

    import speedb_amd as S
    from speedb_amd import _lib
    rnd = random.Random(12)
    lens = [rnd.randrange(1000, 1101) for _ in range(20000)] + [0, 1, 15, 16, 17, 5000, 40000]
    offs = np.cumsum([0] + lens[:-1]).astype(np.uint64)
    src = torch.randint(0, 256, (int(sum(lens)) + 64,), dtype=torch.uint8, device="cuda")
    frags, nf, nbytes, _ = S.wal_plan(offs, lens, 0, False)
    d_frags = torch.frombuffer(bytearray(bytes(frags)[:nf * ctypes.sizeof(S.mck_wal_fragment)]),
                               dtype=torch.uint8).to("cuda")
    G = 4096
    arena = torch.full((G + nbytes + G,), 0xA7, dtype=torch.uint8, device="cuda")
    out = arena[G:G + nbytes]
    crc_arena = torch.full((1024 + nf + 1024,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    crc = crc_arena[1024:1024 + nf]
    _lib.check(_lib.lib.mck_wal_write_batch(src.data_ptr(), d_frags.data_ptr(), nf, 7, crc.data_ptr(),
                                            out.data_ptr(), None), "mck_wal_write_batch")
    torch.cuda.synchronize()
    a = arena.cpu().numpy()
    assert (a[:G] == 0xA7).all() and (a[G + nbytes:] == 0xA7).all()
    c = crc_arena.cpu().numpy()
    assert (c[:1024] == 0x5A5A5A5A).all() and (c[1024 + nf:] == 0x5A5A5A5A).all()
    res = S.wal_verify_batch(out, nbytes, 7).cpu().numpy()
    assert (res[:, 1] == 0).all() and int(res[:, 0].sum()) == nf

"""GPU parity of the host-resident pipeline (mck_host_batch_checksum, row n1 /
BASELINE.json configs[4]): spans in host memory, H2D in double-buffered
chunks, CRC32C / XXH3 on the device, results back to the host -- against the
CPU oracle, bit-exact.  Covers ragged and uniform spans, chunk-straddling
batches, a single span longer than the chunk, MCK_F_MASK, XXH3, every visible
device (ndev = mck_device_count()), pinned and pageable sources, the reuse and
release of the cached per-device staging, and argument errors."""
import ctypes
import random

import numpy as np
import pytest

from formats import splitmix_bytes

pytestmark = pytest.mark.gpu

LENS = [0, 1, 3, 4, 15, 16, 17, 63, 64, 65, 255, 1000, 1023, 1024, 1025, 4095, 4096, 4097, 4300, 8191,
        16384, 16389, 65536, 65541, 100003]


def ragged(seed, lens, gap=64):
    rnd = random.Random(seed)
    offs, pos = [], 0
    for n in lens:
        pos += rnd.randrange(0, gap)
        offs.append(pos)
        pos += n
    return splitmix_bytes(seed, pos + 64), offs


def test_host_crc_ragged_chunk_straddling(gpu, oracle):
    import speedb_amd as S
    lens = LENS * 8
    random.Random(3).shuffle(lens)
    host, offs = ragged(3, lens)
    buf = np.frombuffer(host, dtype=np.uint8)
    want = [oracle.Value(host[o:o + n]) for o, n in zip(offs, lens)]
    # small chunks: many chunks, spans cut at every chunk edge position
    for chunk in (64 << 10, 200 << 10, 0):
        got, secs = S.host_batch_checksum(S.ChecksumType.kCRC32c, buf, offs, lens, chunk_bytes=chunk)
        assert got.tolist() == want, chunk
        assert secs > 0
    gotm, _ = S.host_batch_checksum(S.ChecksumType.kCRC32c, buf, offs, lens, mask=True, chunk_bytes=96 << 10)
    assert gotm.tolist() == [oracle.Mask(v) for v in want]


def test_host_xxh3_ragged(gpu, oracle):
    import speedb_amd as S
    lens = LENS * 4
    random.Random(4).shuffle(lens)
    host, offs = ragged(4, lens)
    got, _ = S.host_batch_checksum(S.ChecksumType.kXXH3, np.frombuffer(host, dtype=np.uint8), offs, lens,
                                   chunk_bytes=128 << 10)
    assert got.tolist() == [oracle.XXH3(host[o:o + n]) for o, n in zip(offs, lens)]


def test_host_uniform_pinned_all_devices(gpu, oracle):
    import speedb_amd as S
    torch = gpu
    block, count = 4300, 3000  # SST-sized blocks (configs[4]), 12.3 MiB
    host = splitmix_bytes(5, block * count + 64)
    pinned = torch.empty(len(host), dtype=torch.uint8, pin_memory=True)
    pinned.copy_(torch.frombuffer(bytearray(host), dtype=torch.uint8))
    ndev = S.device_count()
    assert ndev >= 1
    want = [oracle.Value(host[i * block:(i + 1) * block]) for i in range(count)]
    for nd in (0, ndev):
        got, _ = S.host_batch_checksum(S.ChecksumType.kCRC32c, pinned, stride=block, length=block, count=count,
                                       ndev=nd, chunk_bytes=1 << 20)
        assert got.tolist() == want, nd
    gx, _ = S.host_batch_checksum(S.ChecksumType.kXXH3, pinned, stride=block, length=block, count=count,
                                  ndev=ndev, chunk_bytes=3 << 20)
    for i in range(0, count, 37):
        assert int(gx[i]) == oracle.XXH3(host[i * block:(i + 1) * block]), i


def test_host_span_longer_than_chunk(gpu, oracle):
    import speedb_amd as S
    lens = [100, 3 << 20, 77, (1 << 20) + 5, 0, 4096]
    host, offs = ragged(6, lens, gap=16)
    buf = np.frombuffer(host, dtype=np.uint8)
    got, _ = S.host_batch_checksum(S.ChecksumType.kCRC32c, buf, offs, lens, chunk_bytes=64 << 10)
    assert got.tolist() == [oracle.Value(host[o:o + n]) for o, n in zip(offs, lens)]
    # the staging grew for the long span; a later small-chunk call reuses it
    got2, _ = S.host_batch_checksum(S.ChecksumType.kCRC32c, buf, offs[:2], lens[:2], chunk_bytes=4096)
    assert got2.tolist() == got[:2].tolist()


def test_host_release_and_reuse(gpu, oracle):
    import speedb_amd as S
    from speedb_amd import _lib
    host, offs = ragged(7, [5000] * 50)
    buf = np.frombuffer(host, dtype=np.uint8)
    want = [oracle.Value(host[o:o + 5000]) for o in offs]
    for _ in range(3):
        got, _ = S.host_batch_checksum(S.ChecksumType.kCRC32c, buf, offs, [5000] * 50, chunk_bytes=20000)
        assert got.tolist() == want
        _lib.lib.mck_host_pipeline_release()
    got, _ = S.host_batch_checksum(S.ChecksumType.kCRC32c, buf, offs, [5000] * 50)
    assert got.tolist() == want


def test_host_errors(gpu):
    from speedb_amd import _lib
    L = _lib.lib
    buf = (ctypes.c_uint8 * 4096)()
    out = (ctypes.c_uint32 * 4)()
    offs = (ctypes.c_uint64 * 2)(100, 50)  # decreasing
    lens = (ctypes.c_uint32 * 2)(10, 10)
    assert L.mck_host_batch_checksum(2, buf, None, None, 16, 16, 4, 0, 0, 0, out, None, None) == -1  # kind
    assert L.mck_host_batch_checksum(1, buf, offs, lens, 0, 0, 2, 0, 0, 0, out, None, None) == -1
    assert b"non-decreasing" in L.mck_last_error()
    assert L.mck_host_batch_checksum(1, None, None, None, 16, 16, 4, 0, 0, 0, out, None, None) == -1
    assert L.mck_host_batch_checksum(4, buf, None, None, 16, 16, 4, 0, 0, 0, out, None, None) == -1  # no out64
    # empty batch: nothing to do
    assert L.mck_host_batch_checksum(1, None, None, None, 0, 0, 0, 0, 0, 0, None, None, None) == 0


@pytest.mark.parametrize("k", [2, 4, 8])
def test_host_virtual_devices(gpu, oracle, k):
    """The ndev > 1 branch of mck_host_batch_checksum -- one host thread,
    staging and stream pair per device, concurrent first use, the byte-balanced
    device split (mck_partition_spans) and the result concatenation -- run on
    a one-GPU box through mck_test_set_virtual_devices(k): k "devices" that
    are all device 0.  Ragged spans (CRC32C and XXH3) and 4300-B pinned blocks
    against the oracle; more devices than that is refused."""
    import speedb_amd as S
    from speedb_amd import _lib
    torch = gpu
    L = _lib.lib
    assert L.mck_test_set_virtual_devices(k) == 0
    try:
        lens = LENS * 6
        random.Random(10 + k).shuffle(lens)
        host, offs = ragged(10 + k, lens)
        buf = np.frombuffer(host, dtype=np.uint8)
        got, _ = S.host_batch_checksum(S.ChecksumType.kCRC32c, buf, offs, lens, ndev=k, chunk_bytes=96 << 10)
        assert got.tolist() == [oracle.Value(host[o:o + n]) for o, n in zip(offs, lens)]
        gx, _ = S.host_batch_checksum(S.ChecksumType.kXXH3, buf, offs, lens, ndev=k, chunk_bytes=160 << 10)
        assert gx.tolist() == [oracle.XXH3(host[o:o + n]) for o, n in zip(offs, lens)]
        block, count = 4300, 2000
        hb = splitmix_bytes(20 + k, block * count + 64)
        pinned = torch.empty(len(hb), dtype=torch.uint8, pin_memory=True)
        pinned.copy_(torch.frombuffer(bytearray(hb), dtype=torch.uint8))
        got, _ = S.host_batch_checksum(S.ChecksumType.kCRC32c, pinned, stride=block, length=block, count=count,
                                       ndev=k, mask=True, chunk_bytes=1 << 20)
        assert got.tolist() == [oracle.Mask(oracle.Value(hb[i * block:(i + 1) * block])) for i in range(count)]
        # fewer spans than devices: empty shares
        got, _ = S.host_batch_checksum(S.ChecksumType.kCRC32c, buf, offs[:1], lens[:1], ndev=k)
        assert got.tolist() == [oracle.Value(host[offs[0]:offs[0] + lens[0]])]
        assert L.mck_host_batch_checksum(1, buf.ctypes.data, None, None, 16, 16, 4, 0, k + 1, 0,
                                         (ctypes.c_uint32 * 4)(), None, None) == -3  # MCK_ENODEV
    finally:
        assert L.mck_test_set_virtual_devices(0) == 0

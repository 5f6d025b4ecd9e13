"""XXH3_64bits / XXPH3 of short spans (<= 240 B) on 16-lane rows (round 6,
mck_xxh.hpp x3_short_rows / x3s_row_hash): one 16-byte window per lane and
a half-row reduction replace the one-lane walk of util/xxhash.h:3990-4130
(XXPH3: util/xxph3.h:1086-1147).  Every length 0..260 at every start
alignment, on each driver that hashes short spans:

* the wave kernel's rows share (ragged batches averaging < 2.5 KiB): short
  spans and 241..512-byte spans on lane quads (x3_short_quads,
  x3_mid_quads), longer ones on the row loop,
* the wave kernel's piece path (shares averaging >= 2.5 KiB; short spans
  one per lane),
* the rows kernel (uniform batches, x3_next_long),
* k_xph3 (NPHash64 batches, seeded XXPH3),
* k_wal_recover (records of <= 240 B hashed at their last round).

Bit-exact against the oracle (oracle/oracle.c, pinned by tests/golden)."""
import random

import numpy as np
import pytest

from formats import splitmix_bytes

pytestmark = pytest.mark.gpu


def _pack(torch, seed, lens, aligns=None, gap=16):
    rnd = random.Random(seed)
    offs, pos = [], 0
    for k, n in enumerate(lens):
        pos += rnd.randrange(0, gap)
        if aligns is not None:
            pos += (aligns[k] - pos) % 16
        offs.append(pos)
        pos += n
    host = splitmix_bytes(seed, pos + 64)
    dev = torch.frombuffer(bytearray(host), dtype=torch.uint8).to("cuda")
    return host, dev, offs


def _spans(torch, S, dev, offs, lens):
    return S.Spans(dev, len(offs), offsets=torch.tensor(offs, dtype=torch.int64, device="cuda"),
                   lengths=torch.tensor(lens, dtype=torch.int32, device="cuda"))


def _forced(lib, mode, fn):
    from speedb_amd import _lib
    try:
        _lib.check(lib.mck_test_set_xxh3_driver(mode), "mck_test_set_xxh3_driver")
        return fn()
    finally:
        _lib.check(lib.mck_test_set_xxh3_driver(0), "mck_test_set_xxh3_driver")


def _all_short():
    # every length 0..260 at every alignment mod 16 (a length's 16 copies)
    lens = [n for n in range(261) for _ in range(16)]
    aligns = [a for _ in range(261) for a in range(16)]
    return lens, aligns


@pytest.mark.parametrize("driver", [0, 1, 2])
def test_xxh3_short_every_length_alignment(gpu, oracle, driver):
    """driver 0: the engine's choice (a ragged batch of mostly short spans:
    the wave kernel's rows share, lane quads), 1: the wave kernel, 2: the
    rows kernel."""
    import speedb_amd as S
    from speedb_amd._lib import lib
    torch = gpu
    lens, aligns = _all_short()
    rnd = random.Random(5)
    order = list(range(len(lens)))
    rnd.shuffle(order)
    lens = [lens[k] for k in order]
    aligns = [aligns[k] for k in order]
    host, dev, offs = _pack(torch, 11 + driver, lens, aligns)
    sp = _spans(torch, S, dev, offs, lens)
    got = _forced(lib, driver, lambda: S.xxh3_64_batch(sp)).cpu().numpy().view(np.uint64)
    bad = [(lens[i], offs[i] % 16) for i in range(len(lens))
           if int(got[i]) != oracle.XXH3(host[offs[i]:offs[i] + lens[i]])]
    assert not bad, bad[:10]


def test_xxh3_short_in_rows_share(gpu, oracle):
    """A ragged batch averaging ~600 B (the wave kernel's rows share): the
    short spans go through x3_short_rows before the row loop, the long ones
    through the row loop, every span bit-exact."""
    import speedb_amd as S
    torch = gpu
    rnd = random.Random(17)
    lens = []
    for k in range(20000):
        lens.append(rnd.randrange(0, 241) if k % 3 == 0 else rnd.randrange(241, 1400))
    host, dev, offs = _pack(torch, 23, lens)
    sp = _spans(torch, S, dev, offs, lens)
    got = S.xxh3_64_batch(sp).cpu().numpy().view(np.uint64)
    bad = [i for i in range(len(lens)) if int(got[i]) != oracle.XXH3(host[offs[i]:offs[i] + lens[i]])]
    assert not bad, [(lens[i], offs[i] % 16) for i in bad[:10]]


@pytest.mark.parametrize("length", [0, 1, 3, 4, 8, 9, 16, 17, 32, 33, 64, 65, 96, 97, 128, 129, 143, 144,
                                    200, 239, 240])
def test_xxh3_short_uniform_rows_kernel(gpu, oracle, length):
    """Uniform short batches run on the rows kernel (x3_next_long hashes
    them with the whole row); odd strides put every span at another byte
    alignment."""
    import speedb_amd as S
    torch = gpu
    n = 3000
    stride = length + 5
    host = splitmix_bytes(length + 101, n * stride + 64)
    dev = torch.frombuffer(bytearray(host), dtype=torch.uint8).to("cuda")
    sp = S.Spans(dev, n, offsets=torch.arange(n, dtype=torch.int64, device="cuda") * stride, length=length)
    got = S.xxh3_64_batch(sp).cpu().numpy().view(np.uint64)
    bad = [i for i in range(n) if int(got[i]) != oracle.XXH3(host[i * stride:i * stride + length])]
    assert not bad, bad[:10]


@pytest.mark.parametrize("seed", [0, 0xD28AAD72F49BD50B])
def test_np_hash64_short_every_length(gpu, oracle, seed):
    """Seeded XXPH3 (NPHash64, util/hash.cc:81-88) of every length 0..260
    at every alignment on k_xph3's rows (the short classes key mix16 with
    secret +/- seed)."""
    import speedb_amd as S
    torch = gpu
    lens, aligns = _all_short()
    host, dev, offs = _pack(torch, 31, lens, aligns)
    sp = _spans(torch, S, dev, offs, lens)
    got = S.np_hash64_batch(sp, seed=seed).cpu().numpy().view(np.uint64)
    bad = [(lens[i], offs[i] % 16) for i in range(len(lens))
           if int(got[i]) != oracle.Hash64(host[offs[i]:offs[i] + lens[i]], seed)]
    assert not bad, bad[:10]


def test_wal_recover_every_short_record(gpu, oracle):
    """k_wal_recover hashes records of <= 240 B with the whole row at their
    last round: every payload length 0..260, four times (so the 7-byte
    headers walk the payload through every dword alignment), in one log."""
    import speedb_amd as S
    from test_wal_recover import LOG, WalWriter, _payload, _plan
    torch = gpu
    rng = np.random.default_rng(3)
    lens = list(range(261)) * 4
    rng.shuffle(lens)
    for recycle in (False, True):
        w = WalWriter(oracle, log_number=LOG, recycle=recycle)
        for n in lens:
            w.add_record(_payload(rng, n))
        img = bytes(w.buf)
        d = torch.frombuffer(bytearray(img + bytes(16)), dtype=torch.uint8).cuda()
        plan, dp = _plan(S, torch, img)
        ok, h = S.wal_recover_batch(d, dp, LOG)
        assert (ok.cpu().numpy() == 1).all()
        hv = h.cpu().numpy().view(np.uint64)
        hs = 11 if recycle else 7
        bad = [(n, (off + hs) & 3) for k, (off, t, n) in enumerate(w.records)
               if t in (1, 5) and int(hv[k]) != oracle.XXH3(img[off + hs:off + hs + n])]
        assert not bad, bad[:10]


def test_xxh3_short_in_piece_path(gpu, oracle):
    """Shares averaging >= 2.5 KiB run on the wave units (the piece path),
    whose short spans are hashed one per lane before the pieces: every
    length 0..260 between 6-9 KiB spans, each span bit-exact."""
    import speedb_amd as S
    torch = gpu
    rnd = random.Random(61)
    lens = []
    for n in range(261):
        lens += [n, rnd.randrange(6000, 9000)]
    host, dev, offs = _pack(torch, 67, lens)
    sp = _spans(torch, S, dev, offs, lens)
    got = S.xxh3_64_batch(sp).cpu().numpy().view(np.uint64)
    bad = [(lens[i], offs[i] % 16) for i in range(len(lens))
           if int(got[i]) != oracle.XXH3(host[offs[i]:offs[i] + lens[i]])]
    assert not bad, bad[:10]


@pytest.mark.parametrize("quads", [1, 0])
def test_np_hash64_uniform_short_quads(gpu, oracle, quads):
    """Uniform XXPH3 batches of <= 240-byte spans run on k_xph3_quads (one
    span per lane quad; the test hook sends them to the row driver for the
    comparison): every length 0..240, odd strides, two seeds."""
    import speedb_amd as S
    from speedb_amd import _lib
    torch = gpu
    try:
        _lib.check(_lib.lib.mck_test_set_xph3_quads(quads), "mck_test_set_xph3_quads")
        for seed in (0, 0xA5155AE5E937AA16):
            bad = []
            for length in range(0, 241, 3 if quads == 0 else 1):
                n = 700
                stride = length + 7
                host = splitmix_bytes(length * 31 + 5, n * stride + 64)
                dev = torch.frombuffer(bytearray(host), dtype=torch.uint8).to("cuda")
                sp = S.Spans(dev, n, offsets=torch.arange(n, dtype=torch.int64, device="cuda") * stride,
                             length=length)
                got = S.np_hash64_batch(sp, seed=seed).cpu().numpy().view(np.uint64)
                bad += [(length, i) for i in range(0, n, 37)
                        if int(got[i]) != oracle.Hash64(host[i * stride:i * stride + length], seed)]
            assert not bad, bad[:10]
    finally:
        _lib.check(_lib.lib.mck_test_set_xph3_quads(1), "mck_test_set_xph3_quads")


@pytest.mark.parametrize("vlen", [0, 5, 16, 17, 100, 128, 129, 200, 240])
def test_kv_protect_uniform_short_values(gpu, oracle, vlen):
    """Per-KV protection (db/kv_checksum.h ProtectKV / ProtectKVO /
    ProtectKVOS) of uniform short values on the lane quads: the epilogue
    (key, op type, seqno hashes) runs on each quad's lane 0; against the
    oracle's KvProtect for every mode, and verify flags exactly the
    corrupted entries."""
    import speedb_amd as S
    torch = gpu
    n, kb = 3000, 24
    host_k = splitmix_bytes(vlen + 1, n * kb + 64)
    host_v = splitmix_bytes(vlen + 2, n * max(vlen, 1) + 64)
    keys = torch.frombuffer(bytearray(host_k), dtype=torch.uint8).to("cuda")
    vals = torch.frombuffer(bytearray(host_v), dtype=torch.uint8).to("cuda")
    ks = S.Spans.uniform(keys, kb, n)
    vs = S.Spans(vals, n, stride=vlen, length=vlen)
    rnd = random.Random(vlen)
    ops = torch.tensor([rnd.randrange(256) for _ in range(n)], dtype=torch.uint8, device="cuda")
    seqs = torch.tensor([rnd.randrange(1 << 56) for _ in range(n)], dtype=torch.int64, device="cuda")
    for mode, extra in ((S.ProtectionKind.KV, None), (S.ProtectionKind.KVO, None), (S.ProtectionKind.KVOS, seqs)):
        out = S.kv_protect_batch(mode, ks, vs, ops, extra)
        got = out.cpu().numpy().view(np.uint64)
        o = ops.cpu().tolist()
        ex = seqs.cpu().tolist()
        for i in range(0, n, 53):
            k = host_k[i * kb:(i + 1) * kb]
            v = host_v[i * vlen:(i + 1) * vlen] if vlen else b""
            want = oracle.KvProtect(int(mode), k, v, o[i], ex[i] if extra is not None else 0)
            assert int(got[i]) == want, (int(mode), i)

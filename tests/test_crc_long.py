"""The body/head CRC driver (mck_crc_bh.hpp, in k_crc_ragged) against the oracle.

A workgroup whose share averages more than 2.5 KiB per span takes it on the
body/head driver: each span's whole 4 KiB rounds (ending at its 16-aligned
end) in pieces of at most four rounds, its head (the rest, or the whole of
a short span) on 4-lane rows 16 heads at a time (one lane per head when
the window's heads are short), the parts joined in an
LDS accumulator (moved to the span end by zshift(4096 m)).  The cases below
are the shapes that stress it: SST data blocks (4096 + 0..255 bytes + the
type byte, never 16-aligned), uniform non-aligned strides, every span length
around the round / piece / head-batch boundaries, long spans (many pieces
finishing on different waves), runs of empty spans, many windows, non-zero
Extend inits.  The driver forced on every generic CRC test (short spans,
WAL, blob) and these tests with the row drivers: test_crc_rows.py
test_auto_kernel_forced_drivers_subprocess.  Bit-exact throughout."""
import random
import struct

import numpy as np
import pytest

from formats import splitmix_bytes, sst_blocks

pytestmark = pytest.mark.gpu


def _u32(t):
    return t.cpu().numpy().view(np.uint32).astype(np.uint64).tolist()


def _pack(torch, seed, lens, gap=64):
    rnd = random.Random(seed)
    offs, pos = [], 0
    for n in lens:
        pos += rnd.randrange(0, gap)
        offs.append(pos)
        pos += n
    host = splitmix_bytes(seed, pos + 64)
    dev = torch.frombuffer(bytearray(host), dtype=torch.uint8).to("cuda")
    return host, dev, offs


def _spans(torch, S, dev, offs, lens):
    return S.Spans(dev, len(offs), offsets=torch.tensor(offs, dtype=torch.int64, device="cuda"),
                   lengths=torch.tensor(lens, dtype=torch.int32, device="cuda"))


def test_long_sst_block_shapes(gpu, oracle):
    """40K spans of 4096 + 0..255 (+1) bytes at every alignment: the 5-unit
    blocks whose last unit shares a wave iteration with the next block."""
    import speedb_amd as S
    torch = gpu
    rnd = random.Random(5)
    lens = [4096 + rnd.randrange(0, 256) + 1 for _ in range(40_000)]
    host, dev, offs = _pack(torch, 5, lens)
    sp = _spans(torch, S, dev, offs, lens)
    got = _u32(S.crc32c_batch(sp))
    masked = _u32(S.crc32c_batch(sp, mask=True))
    inits = [rnd.getrandbits(32) for _ in lens]
    ext = _u32(S.crc32c_batch(sp, init_crcs=torch.tensor(np.array(inits, dtype=np.uint32).view(np.int32),
                                                          device="cuda")))
    for i in range(0, len(lens), 7):
        o, n = offs[i], lens[i]
        d = host[o:o + n]
        v = oracle.Value(d)
        assert got[i] == v, (i, o, n)
        assert masked[i] == oracle.Mask(v), (i, o, n)
        assert ext[i] == oracle.Extend(inits[i], d), (i, o, n)


@pytest.mark.parametrize("stride", [4300, 4101, 5000, 8193])
def test_long_uniform_unaligned_stride(gpu, oracle, stride):
    """Uniform batches whose length is not a 16-byte multiple (implicit
    offsets i * stride): the body/head driver, not the aligned uniform kernel."""
    import speedb_amd as S
    torch = gpu
    count = 30_000
    host = splitmix_bytes(stride, count * stride + 64)
    dev = torch.frombuffer(bytearray(host), dtype=torch.uint8).to("cuda")
    got = _u32(S.crc32c_batch(S.Spans.uniform(dev, stride, count)))
    for i in list(range(0, count, 97)) + [count - 1]:
        assert got[i] == oracle.Value(host[i * stride:(i + 1) * stride]), i


def test_long_boundary_lengths(gpu, oracle):
    """Lengths around the 1 KiB unit, the 4-unit iteration and multiples of
    16 units, at every start alignment, mixed with 3-8 KiB spans so the
    workgroups choose the body/head driver."""
    import speedb_amd as S
    torch = gpu
    rnd = random.Random(11)
    special = []
    for u in (1, 2, 3, 4, 5, 8, 16, 17, 23, 24, 25, 26, 40, 41, 48, 49, 64, 65, 100, 257):
        for d in (-17, -16, -15, -1, 0, 1, 15, 16, 17):
            special.append(max(0, 1024 * u + d))
    lens = special + [rnd.randrange(3000, 8000) for _ in range(3000)]
    rnd.shuffle(lens)
    host, dev, offs = _pack(torch, 11, lens)
    sp = _spans(torch, S, dev, offs, lens)
    inits = [rnd.getrandbits(32) for _ in lens]
    got = _u32(S.crc32c_batch(sp))
    ext = _u32(S.crc32c_batch(sp, init_crcs=torch.tensor(np.array(inits, dtype=np.uint32).view(np.int32),
                                                          device="cuda")))
    for i, (o, n) in enumerate(zip(offs, lens)):
        d = host[o:o + n]
        assert got[i] == oracle.Value(d), (i, o, n)
        assert ext[i] == oracle.Extend(inits[i], d), (i, o, n)


def test_long_long_spans_split(gpu, oracle):
    """Spans of 25 units to 4 MiB (a 4 MiB span is longer than a whole
    window's stream: shared by all 16 waves), empty spans and short spans in
    between."""
    import speedb_amd as S
    torch = gpu
    rnd = random.Random(23)
    lens = [25 * 1024 + 3, 65536 + 255, 200_000, 1 << 20, (4 << 20) + 7, 0, 5, 1000, 0]
    lens += [rnd.randrange(20_000, 300_000) for _ in range(300)]
    rnd.shuffle(lens)
    host, dev, offs = _pack(torch, 23, lens)
    sp = _spans(torch, S, dev, offs, lens)
    inits = [rnd.getrandbits(32) for _ in lens]
    got = _u32(S.crc32c_batch(sp))
    ext = _u32(S.crc32c_batch(sp, init_crcs=torch.tensor(np.array(inits, dtype=np.uint32).view(np.int32),
                                                          device="cuda")))
    for i, (o, n) in enumerate(zip(offs, lens)):
        d = host[o:o + n]
        assert got[i] == oracle.Value(d), (i, o, n)
        assert ext[i] == oracle.Extend(inits[i], d), (i, o, n)


def test_long_runs_of_empty_spans(gpu, oracle):
    """Runs of 0..200 empty spans between 3-9 KiB spans: a stream's lookahead
    over the units' prefix passes more than 63 empty spans at once."""
    import speedb_amd as S
    torch = gpu
    rnd = random.Random(57)
    lens = []
    for _ in range(600):
        lens += [0] * rnd.choice([0, 0, 1, 5, 63, 64, 65, 130, 200])
        lens.append(rnd.randrange(3000, 9000))
    host, dev, offs = _pack(torch, 57, lens, gap=8)
    sp = _spans(torch, S, dev, offs, lens)
    inits = [rnd.getrandbits(32) for _ in lens]
    got = _u32(S.crc32c_batch(sp))
    ext = _u32(S.crc32c_batch(sp, init_crcs=torch.tensor(np.array(inits, dtype=np.uint32).view(np.int32),
                                                          device="cuda")))
    for i, (o, n) in enumerate(zip(offs, lens)):
        d = host[o:o + n]
        assert got[i] == oracle.Value(d), (i, o, n)
        assert ext[i] == oracle.Extend(inits[i], d), (i, o, n)


def test_long_many_windows(gpu, oracle):
    """More spans per workgroup than one LDS descriptor window (832): the
    share is processed in several windows, and in several launches."""
    import speedb_amd as S
    torch = gpu
    rnd = random.Random(31)
    lens = np.array([rnd.randrange(2600, 3400) for _ in range(420_000)], dtype=np.int64)
    offs = np.concatenate([[0], np.cumsum(lens + 3)[:-1]])
    total = int(offs[-1] + lens[-1] + 64)
    g = torch.Generator(device="cuda")
    g.manual_seed(31)
    dev = torch.randint(0, 256, (total,), dtype=torch.uint8, device="cuda", generator=g)
    sp = S.Spans(dev, len(lens), offsets=torch.tensor(offs, dtype=torch.int64, device="cuda"),
                 lengths=torch.tensor(lens.astype(np.int32), device="cuda"))
    got = _u32(S.crc32c_batch(sp))
    for i in list(range(0, len(lens), 1009)) + [len(lens) - 1]:
        o, n = int(offs[i]), int(lens[i])
        assert got[i] == oracle.Value(bytes(dev[o:o + n].cpu().numpy())), (i, o, n)


@pytest.mark.parametrize("ctype", [1, 4])
def test_long_sst_verify_mix(gpu, oracle, ctype):
    """VerifyBlockChecksum over a compaction mix of 4/16/64 KiB blocks with
    jitter (64 KiB blocks cut by stream boundaries: the epilogue runs on
    whichever wave finishes the last part -- the CRC body/head driver, and for
    kXXH3 the wave driver's pieces), context checksums, then flipped bytes."""
    import speedb_amd as S
    torch = gpu
    rnd = random.Random(77)
    sizes = [rnd.choice([4096] * 6 + [16384] * 3 + [65536]) + rnd.randrange(0, 256) for _ in range(2000)]
    payloads = [splitmix_bytes(5000 + i, n) for i, n in enumerate(sizes)]
    comps = [rnd.choice([0, 1, 7]) for _ in sizes]
    base_ctx = 0x5EED1234
    file_start = 12345
    img, offs, lens = sst_blocks(oracle, payloads, ctype, comps, base_ctx, file_start)
    dev = torch.frombuffer(bytearray(img + bytes(64)), dtype=torch.uint8).to("cuda")
    sp = _spans(torch, S, dev, offs, lens)
    foff = torch.tensor([file_start + o for o in offs], dtype=torch.int64, device="cuda")
    ct = torch.tensor(comps, dtype=torch.uint8, device="cuda")
    tr = _u32(S.sst_trailer_batch(ctype, sp, ct, file_offsets=foff, base_context_checksum=base_ctx))
    for i, o in enumerate(offs):
        assert tr[i] == struct.unpack_from("<I", img, o + lens[i] + 1)[0], (i, lens[i])
    mm, comp, stored, cnt = S.sst_verify_batch(ctype, sp, file_offsets=foff, base_context_checksum=base_ctx)
    assert int(cnt.item()) == 0 and int(mm.sum().item()) == 0
    bad = sorted(rnd.sample(range(len(sizes)), 25))
    cor = bytearray(img)
    for i in bad:
        cor[offs[i] + rnd.randrange(0, lens[i] + 5)] ^= 1 << rnd.randrange(8)
    dev2 = torch.frombuffer(bytearray(bytes(cor) + bytes(64)), dtype=torch.uint8).to("cuda")
    mm, comp, stored, cnt = S.sst_verify_batch(ctype, _spans(torch, S, dev2, offs, lens), file_offsets=foff,
                                               base_context_checksum=base_ctx)
    assert [i for i, v in enumerate(mm.cpu().tolist()) if v] == bad
    assert int(cnt.item()) == len(bad)




@pytest.mark.parametrize("ctype", [1, 4])
def test_sst_mix_oracle_at_scale(gpu, oracle, ctype):
    """configs[2]'s shape at scale: ~256 MiB of 4/16/64 KiB + jitter blocks
    at byte offsets (a compaction's input), every trailer sealed by the
    ORACLE (the reference's BuiltinChecksumWithLastByte + context modifier,
    not the engine's write kernel), then one verify batch: no block may
    mismatch and every computed checksum must equal the oracle's stored one
    -- bit-exact parity over ~18K blocks, 10x the mix test above."""
    import speedb_amd as S
    torch = gpu
    rnd = random.Random(4242 + ctype)
    sizes, total = [], 0
    while total < (256 << 20):
        n = rnd.choice([4096] * 6 + [16384] * 3 + [65536]) + rnd.randrange(0, 256)
        sizes.append(n)
        total += n
    pool = splitmix_bytes(7000 + ctype, total)
    comps = [rnd.choice([0, 1, 7]) for _ in sizes]
    base_ctx, file_start = 0x1234ABCD, 4096 + 13
    img = bytearray()
    offs, pos = [], 0
    want = []
    for n, ct in zip(sizes, comps):
        p = pool[pos:pos + n]
        pos += n
        off = len(img)
        raw = oracle.BuiltinLast(ctype, p, ct)
        ck = (raw + oracle.ContextModifier(base_ctx, file_start + off)) & 0xFFFFFFFF
        offs.append(off)
        want.append(raw)  # computed = the builtin checksum, context removed (format.h:119)
        img += p + bytes([ct]) + struct.pack("<I", ck)
    dev = torch.frombuffer(img + bytes(64), dtype=torch.uint8).to("cuda")
    sp = _spans(torch, S, dev, offs, sizes)
    foff = torch.tensor([file_start + o for o in offs], dtype=torch.int64, device="cuda")
    mm, comp, stored, cnt = S.sst_verify_batch(ctype, sp, file_offsets=foff, base_context_checksum=base_ctx)
    assert int(cnt.item()) == 0 and int(mm.sum().item()) == 0
    comp = _u32(comp)
    bad = [i for i in range(len(sizes)) if int(comp[i]) != want[i]]
    assert not bad, bad[:10]


@pytest.mark.parametrize("lo,hi", [(241, 700), (300, 700), (1000, 3000), (2400, 2700), (100, 5000)])
def test_xxh3_ragged_rows_in_wave_kernel(gpu, oracle, lo, hi):
    """XXH3 over ragged batches whose shares average 256 B - 2.5 KiB run on
    16-lane rows inside the wave kernel (x3_share_rows, round 5); around and
    across the bounds, every span's XXH3_64bits against the oracle, spans at
    byte offsets, some short (<= 240 B) ones mixed in for the wide shape."""
    import speedb_amd as S
    torch = gpu
    rnd = random.Random(lo * 7 + hi)
    n = 12000
    lens = [rnd.randrange(lo, hi + 1) for _ in range(n)]
    offs, pos = [], 0
    for ln in lens:
        offs.append(pos)
        pos += ln + rnd.randrange(0, 9)
    host = splitmix_bytes(lo + hi, pos + 64)
    dev = torch.frombuffer(bytearray(host), dtype=torch.uint8).to("cuda")
    sp = _spans(torch, S, dev, offs, lens)
    got = S.xxh3_64_batch(sp).cpu().numpy().view(np.uint64)
    bad = [i for i in range(n) if int(got[i]) != oracle.XXH3(host[offs[i]:offs[i] + lens[i]])]
    assert not bad, bad[:10]


@pytest.mark.parametrize("length", [3072, 16384])
def test_xxh3_uniform_long_spans_on_wave_kernel(gpu, oracle, length):
    """Uniform XXH3 batches of >= 3 KiB spans (and >= 16 per CU) run on the
    wave kernel since round 5 (kX3UniformWaveMin): every span against the
    oracle, and the same batch on the rows kernel (test hook) agrees."""
    import speedb_amd as S
    from speedb_amd import _lib
    torch = gpu
    n = 16 * torch.cuda.get_device_properties(0).multi_processor_count + 17
    host = splitmix_bytes(length, n * length)
    dev = torch.frombuffer(bytearray(host + bytes(64)), dtype=torch.uint8).to("cuda")
    sp = S.Spans.uniform(dev, length, n)
    got = S.xxh3_64_batch(sp).cpu().numpy().view(np.uint64)
    bad = [i for i in range(n) if int(got[i]) != oracle.XXH3(host[i * length:(i + 1) * length])]
    assert not bad, bad[:10]
    try:
        _lib.check(_lib.lib.mck_test_set_xxh3_driver(2), "mck_test_set_xxh3_driver")
        rows = S.xxh3_64_batch(sp).cpu().numpy().view(np.uint64)
    finally:
        _lib.check(_lib.lib.mck_test_set_xxh3_driver(0), "mck_test_set_xxh3_driver")
    assert (rows == got).all()


@pytest.mark.parametrize("length", [1000, 1024, 1025, 1032, 1040, 1088, 2048, 2056])
def test_xxh3_rows_load_policy_by_alignment(gpu, oracle, length):
    """The XXH3 / XXPH3 row loop runs one of two instances per wave --
    non-temporal loads when every row's first span is 16-byte aligned, the
    default policy otherwise (xxh3_rows_loop, round 5): uniform batches whose
    spans are all aligned (1024, 2048), alternate (1000, 2056: 8-byte steps)
    or mostly misaligned (1025, 1032, 1040, 1088), on the rows kernel,
    against the oracle; and per-KV protection of values at the same stride
    (XXPH3, kind 2).  1025-1088 and 2056 (XXH3) and 1024, 1040, 1088, 2048,
    2056 (XXPH3) end in a segment with no stripe, finished in the iteration
    of the full segment before it."""
    import speedb_amd as S
    torch = gpu
    n = 3000
    host = splitmix_bytes(length + 5, n * length)
    dev = torch.frombuffer(bytearray(host + bytes(64)), dtype=torch.uint8).to("cuda")
    sp = S.Spans.uniform(dev, length, n)
    got = S.xxh3_64_batch(sp).cpu().numpy().view(np.uint64)
    bad = [i for i in range(n) if int(got[i]) != oracle.XXH3(host[i * length:(i + 1) * length])]
    assert not bad, bad[:10]
    kb = 16
    keys = splitmix_bytes(length + 6, n * kb)
    kd = torch.frombuffer(bytearray(keys + bytes(64)), dtype=torch.uint8).to("cuda")
    ks = S.Spans.uniform(kd, kb, n)
    ops = [(7 * i) % 256 for i in range(n)]
    ex = [(0x9E3779B97F4A7C15 * (i + 3)) & (2 ** 64 - 1) for i in range(n)]
    dops = torch.tensor(ops, dtype=torch.uint8, device="cuda")
    dex = torch.tensor(np.array(ex, dtype=np.uint64).view(np.int64), device="cuda")
    kv = S.kv_protect_batch(2, ks, sp, dops, dex).cpu().numpy().view(np.uint64)
    bad = [i for i in range(0, n, 7)
           if int(kv[i]) != oracle.KvProtect(2, keys[i * kb:(i + 1) * kb], host[i * length:(i + 1) * length],
                                             ops[i], ex[i])]
    assert not bad, bad[:10]


@pytest.mark.parametrize("ctype", [1, 4])
@pytest.mark.parametrize("order", ["file", "shuffled", "reversed"])
def test_byte_shares_partition_any_order(gpu, oracle, ctype, order):
    """Byte-balanced workgroup shares (share_by_bytes: the sampled multi-level
    search; k_crc_ragged for SST blocks, k_xxh3_wave) must partition every
    batch -- each span verified exactly once -- whatever the offsets' order:
    file order (exact byte balance), shuffled and reversed (the search is
    only monotone then, the clamp to count shares bounds the imbalance).
    30,000 blocks (> 64 per workgroup, so the byte shares are on), outputs
    pre-filled with sentinels so a span no workgroup visited shows."""
    import speedb_amd as S
    torch = gpu
    rnd = random.Random(900 + ctype)
    n = 30000
    sizes = [rnd.choice([rnd.randrange(200, 3000)] * 19 + [65536 + rnd.randrange(0, 256)]) for _ in range(n)]
    offs, pos = [], 0
    for ln in sizes:
        offs.append(pos)
        pos += ln + 5 + rnd.randrange(0, 3)
    host = bytearray(splitmix_bytes(31 + ctype, pos + 64))
    dev = torch.frombuffer(host, dtype=torch.uint8).to("cuda")
    perm = list(range(n))
    if order == "shuffled":
        rnd.shuffle(perm)
    elif order == "reversed":
        perm.reverse()
    po = [offs[i] for i in perm]
    pl = [sizes[i] for i in perm]
    sp = _spans(torch, S, dev, po, pl)
    ct = torch.zeros(n, dtype=torch.uint8, device="cuda")
    tr = S.sst_trailer_batch(ctype, sp, ct)
    # seal every block on the device: [type 0][LE32 trailer]
    pos_t = torch.tensor(po, dtype=torch.int64, device="cuda") + torch.tensor(pl, dtype=torch.int64, device="cuda")
    trailer = torch.zeros((n, 5), dtype=torch.uint8, device="cuda")
    trailer[:, 1:] = tr.view(torch.uint8).view(n, 4)
    dev[(pos_t.unsqueeze(1) + torch.arange(5, device="cuda")).flatten()] = trailer.flatten()
    # the trailers of a sample against the oracle
    img = bytes(dev.cpu().numpy().tobytes())
    for k in rnd.sample(range(n), 200):
        o, ln = po[k], pl[k]
        assert oracle.BuiltinLast(ctype, img[o:o + ln], 0) == _u32(tr[k:k + 1])[0], (order, k)
    mm = torch.full((n,), 0xAB, dtype=torch.uint8, device="cuda")
    comp = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    stored = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    mm, comp, stored, cnt = S.sst_verify_batch(ctype, sp, outs=(mm, comp, stored))
    assert int(cnt.item()) == 0 and int((mm != 0).sum().item()) == 0, order
    assert torch.equal(comp, stored) and torch.equal(comp, tr)
    bad = sorted(rnd.sample(range(n), 40))
    for k in bad:
        dev[po[k] + rnd.randrange(0, pl[k])] ^= 0x08
    mm, comp, stored, cnt = S.sst_verify_batch(ctype, sp)
    assert torch.nonzero(mm).flatten().cpu().tolist() == bad and int(cnt.item()) == len(bad)

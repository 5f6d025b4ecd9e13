"""GPU parity: every batched entry point of the C ABI against the CPU oracle,
bit-exact, on seeded inputs -- ragged and unaligned spans, every length class
of XXH3, multi-round CRC spans, empty and tiny spans, and the reference's own
known-answer vectors pushed through the device path."""
import random
import struct

import numpy as np
import pytest

from formats import WalWriter, folly_buffer, sst_blocks, splitmix_bytes, wal_expected_blocks

pytestmark = pytest.mark.gpu

LENGTHS = (list(range(0, 70)) + [127, 128, 129, 239, 240, 241, 255, 256, 257, 1023, 1024, 1025,
                                 1087, 1088, 2048, 4032, 4095, 4096, 4097, 4111, 8191, 8192, 8193,
                                 16383, 16384, 16385, 32761, 32762, 65535, 65536, 65537, 100003,
                                 262144, 300001])


def u32(t):
    return t.cpu().numpy().view(np.uint32).astype(np.uint64).tolist()


def u64(t):
    return t.cpu().numpy().view(np.uint64).tolist()


def make_batch(torch, seed, lengths, align_mix=True, pad=4096):
    """Pack spans back to back with random 0..63 byte gaps (so starts are at
    every alignment); returns (host bytes, device tensor, offsets, lengths)."""
    rnd = random.Random(seed)
    offs, pos = [], 0
    for n in lengths:
        pos += rnd.randrange(0, 64) if align_mix else 0
        offs.append(pos)
        pos += n
    total = pos + pad
    host = splitmix_bytes(seed, total)
    dev = torch.frombuffer(bytearray(host), dtype=torch.uint8).to("cuda")
    return host, dev, offs, list(lengths)


def spans(torch, S, dev, offs, lens):
    o = torch.tensor(offs, dtype=torch.int64, device="cuda")
    l_ = torch.tensor(lens, dtype=torch.int32, device="cuda")
    return S.Spans(dev, len(offs), offsets=o, lengths=l_)


def test_crc32c_batch_ragged(gpu, oracle):
    import speedb_amd as S
    torch = gpu
    lens = LENGTHS * 3
    random.Random(1).shuffle(lens)
    host, dev, offs, lens = make_batch(torch, 1, lens)
    sp = spans(torch, S, dev, offs, lens)
    got = u32(S.crc32c_batch(sp))
    torch.cuda.synchronize()
    for i, (o, n) in enumerate(zip(offs, lens)):
        assert got[i] == oracle.Value(host[o:o + n]), (i, o, n)
    gotm = u32(S.crc32c_batch(sp, mask=True))
    for i, (o, n) in enumerate(zip(offs, lens)):
        assert gotm[i] == oracle.Mask(oracle.Value(host[o:o + n]))
    rnd = random.Random(2)
    inits = [rnd.getrandbits(32) for _ in lens]
    it = torch.tensor(np.array(inits, dtype=np.uint32).view(np.int32), device="cuda")
    gote = u32(S.crc32c_batch(sp, init_crcs=it))
    for i, (o, n) in enumerate(zip(offs, lens)):
        assert gote[i] == oracle.Extend(inits[i], host[o:o + n]), (i, n)


def test_crc32c_uniform_blocks(gpu, oracle):
    import speedb_amd as S
    torch = gpu
    # 16-byte multiples take the uniform fast path (full 4 KiB rounds or not)
    for block in (4096, 16384, 65536, 32768, 16, 48, 1008, 4112, 5008, 4100, 1000):
        count = max(1, (8 << 20) // block)
        host = splitmix_bytes(block, block * count)
        dev = torch.frombuffer(bytearray(host), dtype=torch.uint8).to("cuda")
        got = u32(S.crc32c_batch(S.Spans.uniform(dev, block, count)))
        for i in list(range(0, count, max(1, count // 97))) + [count - 1]:
            assert got[i] == oracle.Value(host[i * block:(i + 1) * block]), (block, i)


def test_crc32c_known_answers_on_device(gpu, golden):
    import speedb_amd as S
    torch = gpu
    kat = golden["kat"]
    buf = folly_buffer(kat["folly_buffer_bytes"])
    dev = torch.frombuffer(bytearray(buf), dtype=torch.uint8).to("cuda")
    offs = [o for o, _, _ in kat["folly"]]
    lens = [n for _, n, _ in kat["folly"]]
    got = u32(S.crc32c_batch(spans(torch, S, dev, offs, lens)))
    for g, (_, _, exp) in zip(got, kat["folly"]):
        assert g == (~exp) & 0xFFFFFFFF
    rfc = {r["pattern"]: int(r["crc"], 16) for r in kat["rfc3720"]}
    assert S.crc32c.Value(bytes(32)) == rfc["zeros32"]
    assert S.crc32c.Value(b"\xff" * 32) == rfc["ff32"]
    assert S.crc32c.Value(bytes(range(32))) == rfc["inc32"]
    assert S.crc32c.Value(bytes(31 - i for i in range(32))) == rfc["dec32"]
    assert S.crc32c.Value(bytes.fromhex(kat["iscsi48"])) == rfc["iscsi48"]


def test_scalar_shims(gpu, oracle, golden):
    import speedb_amd as S
    blob = golden["blob"]
    for c in golden["cases"]:
        d = blob[c["off"]:c["off"] + c["len"]]
        assert S.crc32c.Value(d) == c["crc32c"]
        assert S.crc32c.Extend(c["extend_init"], d) == c["crc32c_extend"]
        assert S.XXH3_64bits(d) == c["xxh3"]
        for t, v in c["builtin"].items():
            assert S.ComputeBuiltinChecksum(int(t), d) == v, (t, c["len"])
            if d:
                assert S.ComputeBuiltinChecksumWithLastByte(int(t), d[:-1], d[-1]) == v
    # util/crc32c_test.cc:113-126
    assert S.crc32c.Value(b"hello world") == S.crc32c.Extend(S.crc32c.Value(b"hello "), b"world")
    assert S.crc32c.Crc32cCombine(S.crc32c.Value(b"hello "), S.crc32c.Value(b"world"), 5) == \
        S.crc32c.Value(b"hello world")


def test_checksum_schemas_on_device(gpu, golden):
    """table/table_test.cc:2286-2403 through the device path."""
    import speedb_amd as S
    si = golden["kat"]["schemas_inputs"]
    b2 = (si["b2_repeat"] * si["b2_times"] + si["b2_suffix"]).encode()
    cts = [si["compression_last_bytes"][k] for k in ("ct1", "ct2", "ct3")]
    for t, exp in golden["kat"]["schemas"].items():
        t = int(t)
        assert struct.pack("<I", S.ComputeBuiltinChecksum(t, b"")).hex().upper() == exp["empty"]
        for name, data in (("b0", si["b0"].encode()), ("b1", si["b1"].encode()), ("b2", b2)):
            for ct, want in zip(cts, exp[name]):
                d = data[:-1] + bytes([ct])
                got = S.ComputeBuiltinChecksum(t, d)
                assert struct.pack("<I", got).hex().upper() == want, (t, name, ct)


def test_xxh3_batch_all_length_classes(gpu, oracle):
    import speedb_amd as S
    torch = gpu
    lens = LENGTHS + list(range(230, 260)) + [1024 * k + d for k in (1, 2, 3, 4, 5, 8)
                                              for d in (-65, -64, -63, -1, 0, 1, 63, 64, 65)]
    host, dev, offs, lens = make_batch(torch, 3, lens)
    got = u64(S.xxh3_64_batch(spans(torch, S, dev, offs, lens)))
    for i, (o, n) in enumerate(zip(offs, lens)):
        assert got[i] == oracle.XXH3(host[o:o + n]), (i, n, o % 16)


def test_legacy_xxh_batch(gpu, oracle):
    import speedb_amd as S
    torch = gpu
    host, dev, offs, lens = make_batch(torch, 4, LENGTHS)
    sp = spans(torch, S, dev, offs, lens)
    g32 = u32(S.xxh32_batch(sp, seed=7))
    g64 = u64(S.xxh64_batch(sp, seed=9))
    for i, (o, n) in enumerate(zip(offs, lens)):
        d = host[o:o + n]
        assert g32[i] == oracle.XXH32(d, 7), n
        assert g64[i] == oracle.XXH64(d, 9), n


@pytest.mark.parametrize("ctype", [0, 1, 2, 3, 4])
def test_builtin_checksum_batch(gpu, oracle, ctype):
    import speedb_amd as S
    torch = gpu
    host, dev, offs, lens = make_batch(torch, 10 + ctype, LENGTHS)
    sp = spans(torch, S, dev, offs, lens)
    got = u32(S.builtin_checksum_batch(ctype, sp))
    for i, (o, n) in enumerate(zip(offs, lens)):
        assert got[i] == oracle.Builtin(ctype, host[o:o + n]), (ctype, n)
    rnd = random.Random(ctype)
    last = [rnd.choice([0, 1, 7, 0x40, 255]) for _ in lens]
    lt = torch.tensor(last, dtype=torch.uint8, device="cuda")
    got = u32(S.builtin_checksum_batch(ctype, sp, last_bytes=lt))
    for i, (o, n) in enumerate(zip(offs, lens)):
        assert got[i] == oracle.BuiltinLast(ctype, host[o:o + n], last[i]), (ctype, n)


@pytest.mark.parametrize("ctype", [1, 2, 3, 4])
@pytest.mark.parametrize("base_ctx", [0, 0x9E3779B9])
def test_sst_trailer_and_verify(gpu, oracle, ctype, base_ctx):
    """Write side (trailer compute) and read side (VerifyBlockChecksum) over a
    compaction-shaped run of 4/16/64 KiB blocks with jitter, format_version 6
    context checksums, then one flipped byte in some blocks."""
    import speedb_amd as S
    torch = gpu
    rnd = random.Random(ctype * 1000 + base_ctx % 7)
    sizes = [rnd.choice([4096] * 6 + [16384] * 3 + [65536]) + rnd.randrange(0, 256) for _ in range(120)]
    sizes += [0, 1, 2, 3, 4, 5]
    payloads = [splitmix_bytes(1000 + i, n) for i, n in enumerate(sizes)]
    comps = [rnd.choice([0, 1, 7]) for _ in sizes]
    file_start = 1 << 33  # offsets above 4 GiB exercise the upper-32 fold
    img, offs, lens = sst_blocks(oracle, payloads, ctype, comps, base_ctx, file_start)
    dev = torch.frombuffer(bytearray(img + bytes(64)), dtype=torch.uint8).to("cuda")
    sp = spans(torch, S, dev, offs, lens)
    foff = torch.tensor([file_start + o for o in offs], dtype=torch.int64, device="cuda")
    # write side
    ct = torch.tensor(comps, dtype=torch.uint8, device="cuda")
    tr = u32(S.sst_trailer_batch(ctype, sp, ct, file_offsets=foff, base_context_checksum=base_ctx))
    for i, o in enumerate(offs):
        assert tr[i] == struct.unpack_from("<I", img, o + lens[i] + 1)[0], (i, lens[i])
    # read side, clean
    mm, comp, stored, cnt = S.sst_verify_batch(ctype, sp, file_offsets=foff,
                                               base_context_checksum=base_ctx)
    assert int(cnt.item()) == 0 and int(mm.sum().item()) == 0
    comp_l = u32(comp)
    for i, (o, n) in enumerate(zip(offs, lens)):
        assert comp_l[i] == oracle.Builtin(ctype, img[o:o + n + 1])
    # corrupt: flip one byte (payload, type byte or stored checksum) in 10 blocks
    bad = sorted(rnd.sample(range(len(sizes)), 10))
    cor = bytearray(img)
    for i in bad:
        pos = offs[i] + rnd.randrange(0, lens[i] + 5)
        cor[pos] ^= 1 << rnd.randrange(8)
    dev2 = torch.frombuffer(bytearray(bytes(cor) + bytes(64)), dtype=torch.uint8).to("cuda")
    sp2 = spans(torch, S, dev2, offs, lens)
    torch.cuda.synchronize()
    S.statistics(reset=True)
    mm, comp, stored, cnt = S.sst_verify_batch(ctype, sp2, file_offsets=foff,
                                               base_context_checksum=base_ctx)
    flagged = [i for i, v in enumerate(mm.cpu().tolist()) if v]
    assert flagged == bad
    assert int(cnt.item()) == len(bad)
    # statistics.h:451,455 tickers of that one verify batch
    torch.cuda.synchronize()
    stats = S.statistics()
    assert stats["BLOCK_CHECKSUM_COMPUTE_COUNT"] == len(sizes)
    assert stats["BLOCK_CHECKSUM_MISMATCH_COUNT"] == len(bad)
    assert stats["batches"] == 1 and stats["spans"] == len(sizes)
    st = u32(stored)
    for i in bad:
        o, n = offs[i], lens[i]
        exp_stored = (struct.unpack_from("<I", cor, o + n + 1)[0] -
                      oracle.ContextModifier(base_ctx, file_start + o)) & 0xFFFFFFFF
        assert st[i] == exp_stored


def test_verify_block_checksum_status(gpu, oracle):
    """VerifyBlockChecksum's Status and message (reader_common.cc:46-61)."""
    import speedb_amd as S
    payload = b"This is a long block!" * 50
    for t, base in ((1, 0), (4, 0), (1, 0x1234), (4, 0x77)):
        img, offs, lens = sst_blocks(oracle, [payload], t, [1], base, 4096)
        f = S.Footer(S.ChecksumType(t), base)
        assert S.VerifyBlockChecksum(f, img, len(payload), "000012.sst", 4096).ok()
        cor = bytearray(img)
        cor[10] ^= 0x20
        st = S.VerifyBlockChecksum(f, bytes(cor), len(payload), "000012.sst", 4096)
        assert st.IsCorruption()
        m = st.ToString()
        assert m.startswith("Corruption: block checksum mismatch: stored")
        assert ("(context removed)" in m) == bool(base)
        assert m.endswith(f", type = {t}  in 000012.sst offset 4096 size {len(payload)}")


def test_wal_record_crc_batch(gpu, oracle, golden):
    import speedb_amd as S
    torch = gpu
    blob = golden["blob"]
    recs = golden["wal_records"]
    for ln in sorted({r["log_number"] for r in recs}):
        sub = [r for r in recs if r["log_number"] == ln]
        dev = torch.frombuffer(bytearray(blob + bytes(64)), dtype=torch.uint8).to("cuda")
        sp = spans(torch, S, dev, [r["off"] for r in sub], [r["len"] for r in sub])
        types = torch.tensor([r["type"] for r in sub], dtype=torch.uint8, device="cuda")
        got = u32(S.wal_record_crc_batch(sp, types, ln))
        assert got == [r["crc"] for r in sub]


@pytest.mark.parametrize("recycle", [False, True])
def test_wal_verify_batch(gpu, oracle, recycle):
    import speedb_amd as S
    torch = gpu
    rnd = random.Random(42 + recycle)
    w = WalWriter(oracle, log_number=123, recycle=recycle)
    for _ in range(300):
        n = rnd.choice([0, 1, 10, 100, 1000, 5000, 32761, 40000, rnd.randrange(0, 100000)])
        w.add_record(splitmix_bytes(rnd.getrandbits(32), n))
    data = bytes(w.buf)
    dev = torch.frombuffer(bytearray(data + bytes(64)), dtype=torch.uint8).to("cuda")
    res = S.wal_verify_batch(dev, len(data), 123).cpu().tolist()
    exp = wal_expected_blocks(data, 123, oracle)
    assert [tuple(r) for r in res] == exp
    assert all(r[1] == 0 for r in res)
    # corruption: flip bytes in 5 blocks, plus a wrong log number
    cor = bytearray(data)
    nb = len(res)
    for b in rnd.sample(range(nb), min(5, nb)):
        lo = b * 32768
        cor[lo + rnd.randrange(0, min(32768, len(data) - lo))] ^= 0x10
    dev2 = torch.frombuffer(bytearray(bytes(cor) + bytes(64)), dtype=torch.uint8).to("cuda")
    res2 = [tuple(r) for r in S.wal_verify_batch(dev2, len(cor), 123).cpu().tolist()]
    assert res2 == wal_expected_blocks(bytes(cor), 123, oracle)
    res3 = [tuple(r) for r in S.wal_verify_batch(dev, len(data), 124).cpu().tolist()]
    assert res3 == wal_expected_blocks(data, 124, oracle)


@pytest.mark.parametrize("recycle", [False, True])
def test_wal_verify_many_blocks_per_wave(gpu, oracle, recycle):
    """More blocks than waves (the kernel runs at most 16 x CUs waves), so each
    wave walks a chain of blocks and its record pipeline hands over from a
    record that ends a block to the next block's first record, whose header
    and first round it loaded in advance.  Mixed layouts: full blocks,
    records spilling over blocks, several records per block, trailers of
    1..6 bytes; then payload flips (kBadRecordChecksum on the pipelined
    record and on later records of a block), broken first headers of the
    next block (bad length, zero type: the pipeline restarts) and a
    truncated tail."""
    import speedb_amd as S
    torch = gpu
    rnd = random.Random(7 + recycle)
    w = WalWriter(oracle, log_number=99, recycle=recycle)
    pool = splitmix_bytes(1234 + recycle, 1 << 20)
    waves = 16 * torch.cuda.get_device_properties(0).multi_processor_count
    nblocks = waves + 700
    while len(w.buf) < nblocks * 32768:
        kind = rnd.random()
        hs = 11 if recycle else 7
        if kind < 0.45:  # exactly fills the rest of the block
            n = 32768 - (len(w.buf) % 32768) - hs
            n = n if n >= 0 else 0
        elif kind < 0.6:  # leaves a 1..6-byte trailer (skipped)
            n = max(0, 32768 - (len(w.buf) % 32768) - hs - rnd.randrange(1, 7))
        elif kind < 0.8:
            n = rnd.randrange(0, 3000)
        else:
            n = rnd.randrange(30000, 120000)
        off = rnd.randrange(0, len(pool) - 1)
        payload = (pool[off:] + pool)[:n] if n else b""
        w.add_record(payload)
    data = bytes(w.buf)
    nb = (len(data) + 32767) // 32768
    assert nb > waves
    dev = torch.frombuffer(bytearray(data + bytes(64)), dtype=torch.uint8).to("cuda")
    res = [tuple(r) for r in S.wal_verify_batch(dev, len(data), 99).cpu().tolist()]
    assert res == wal_expected_blocks(data, 99, oracle)
    assert all(r[1] == 0 for r in res)
    cor = bytearray(data)
    for b in rnd.sample(range(nb - 1), 60):
        lo = b * 32768
        what = rnd.randrange(4)
        if what == 0:  # payload flip somewhere in the block
            cor[lo + rnd.randrange(16, 32768)] ^= 0x04
        elif what == 1:  # the first header's length beyond the block
            cor[lo + 4], cor[lo + 5] = 0xFF, 0xFF
        elif what == 2:  # zero type, length 0
            cor[lo + 4:lo + 7] = b"\0\0\0"
        else:  # the stored CRC
            cor[lo] ^= 0x80
    cut = len(cor) - rnd.randrange(1, 32768)
    cor = bytes(cor[:cut])
    dev2 = torch.frombuffer(bytearray(cor + bytes(64)), dtype=torch.uint8).to("cuda")
    res2 = [tuple(r) for r in S.wal_verify_batch(dev2, len(cor), 99).cpu().tolist()]
    assert res2 == wal_expected_blocks(cor, 99, oracle)
    assert sum(r[1] != 0 for r in res2) >= 30
    res3 = [tuple(r) for r in S.wal_verify_batch(dev, len(data), 98).cpu().tolist()]
    assert res3 == wal_expected_blocks(data, 98, oracle)


def test_empty_and_zero_inputs(gpu, oracle):
    import speedb_amd as S
    torch = gpu
    dev = torch.zeros(1 << 16, dtype=torch.uint8, device="cuda")
    out = S.crc32c_batch(S.Spans(dev, 0, stride=0, length=0))
    assert out.numel() == 0
    # ChecksumZeroInputs (table_test.cc:2405-2440): zero buffers never give 0
    lens = list(range(0, 2000)) + list(range(2000, 20000, 37))
    sp = spans(torch, S, dev, [0] * len(lens), lens)
    for t in (1, 2, 3, 4):
        got = u32(S.builtin_checksum_batch(t, sp))
        for n, v in zip(lens, got):
            assert v == oracle.Builtin(t, bytes(n))
            assert v != 0 or (t == 4 and n == 0)


def test_full_size_properties(gpu, oracle):
    """1M x 4 KiB (the bench workload): sampled blocks bit-exact, uniform vs
    explicit descriptors identical, and per-block CRCs combine to the CRC of
    the whole buffer (checksum of checksums via Crc32cCombine)."""
    import speedb_amd as S
    torch = gpu
    count, block = 1 << 20, 4096
    g = torch.Generator(device="cuda")
    g.manual_seed(1234)
    dev = torch.randint(0, 256, (count * block,), dtype=torch.uint8, device="cuda", generator=g)
    got = S.crc32c_batch(S.Spans.uniform(dev, block, count))
    offs = torch.arange(count, dtype=torch.int64, device="cuda") * block
    lens = torch.full((count,), block, dtype=torch.int32, device="cuda")
    got2 = S.crc32c_batch(S.Spans(dev, count, offsets=offs, lengths=lens))
    assert torch.equal(got, got2)
    g_l = u32(got)
    rnd = random.Random(5)
    for i in rnd.sample(range(count), 200) + [0, count - 1]:
        blk = dev[i * block:(i + 1) * block].cpu().numpy().tobytes()
        assert g_l[i] == oracle.Value(blk)
    # whole-buffer CRC of a 64 MiB prefix two ways: one span vs combine of blocks
    n = 16384
    whole = u32(S.crc32c_batch(S.Spans(dev, 1, stride=0, length=n * block)))[0]
    acc = 0
    for i in range(n):
        acc = S.crc32c.Crc32cCombine(acc, g_l[i], block)
    assert acc == whole


# ---- per-KV protection: XXPH3 Hash64 / NPHash64 ----

KV_SEEDS = [0, 0xD28AAD72F49BD50B, 0xA5155AE5E937AA16, 0x77A00858DDD37F21, 0x4A2AB5CBD26F542C]


def test_np_hash64_schemas_on_device(gpu, golden):
    """util/hash_test.cc Hash64SmallValueSchema + Hash64LargeValueSchema
    through the device path (every prefix length 0..429 as one batch)."""
    import speedb_amd as S
    torch = gpu
    small = golden["kat"]["hash64_small"]
    blob = b"".join(bytes.fromhex(h) for h, _ in small)
    offs, pos = [], 0
    for h, _ in small:
        offs.append(pos)
        pos += len(h) // 2
    dev = torch.frombuffer(bytearray(blob + bytes(64)), dtype=torch.uint8).to("cuda")
    got = u64(S.np_hash64_batch(spans(torch, S, dev, offs, [len(h) // 2 for h, _ in small])))
    assert got == [int(v) for _, v in small]
    enc = "abcdefghijklmnopqrstuvwxyz123456789ABCDEFGHIJKLMNOPQRSTUVWXYZ"
    for rep, want in golden["kat"]["hash64_descriptors"].items():
        inp = (rep * 430)[:430].encode()
        dev = torch.frombuffer(bytearray(inp + bytes(64)), dtype=torch.uint8).to("cuda")
        h = u64(S.np_hash64_batch(spans(torch, S, dev, [0] * 430, list(range(430)))))
        assert "".join(enc[x % 61] for x in h) == want, rep


def test_np_hash64_batch_vs_oracle(gpu, oracle, golden):
    import speedb_amd as S
    torch = gpu
    blob = golden["blob"]
    dev = torch.frombuffer(bytearray(blob + bytes(64)), dtype=torch.uint8).to("cuda")
    by_seed = {}
    for c in golden["hash64"]:
        by_seed.setdefault(c["seed"], []).append(c)
    for seed, cs in by_seed.items():
        got = u64(S.np_hash64_batch(spans(torch, S, dev, [c["off"] for c in cs], [c["len"] for c in cs]),
                                    seed))
        assert got == [c["out"] for c in cs], seed
    # every length class, every alignment, long spans with partial/full
    # segments and len % 64 == 0 (no last stripe in the preview)
    lens = LENGTHS + [1024 * k for k in (2, 3, 7)] + [64 * k for k in (5, 17, 33)]
    host, dev2, offs, lens = make_batch(torch, 77, lens)
    for seed in KV_SEEDS + [random.Random(3).getrandbits(64)]:
        got = u64(S.np_hash64_batch(spans(torch, S, dev2, offs, lens), seed))
        for o, n, g in zip(offs, lens, got):
            assert g == oracle.Hash64(host[o:o + n], seed), (n, seed)
    assert S.NPHash64(b"RocksDB", 0) == oracle.Hash64(b"RocksDB")
    assert S.Hash64(host[:5000], 12345) == oracle.Hash64(host[:5000], 12345)


def _kv_batch(torch, S, seed, count):
    rnd = random.Random(seed)
    klen = [rnd.choice([0, 1, 8, 16, 24, 100, 241, rnd.randrange(0, 400)]) for _ in range(count)]
    vlen = [rnd.choice([0, 3, 16, 100, 240, 241, 1000, 1024, 2048, rnd.randrange(0, 5000)])
            for _ in range(count)]
    kh, kd, ko, _ = make_batch(torch, seed, klen)
    vh, vd, vo, _ = make_batch(torch, seed + 1, vlen)
    ops = [rnd.randrange(0, 256) for _ in range(count)]
    ex = [rnd.getrandbits(64) for _ in range(count)]
    return (kh, vh, ko, vo, klen, vlen, ops, ex, spans(torch, S, kd, ko, klen), spans(torch, S, vd, vo, vlen),
            torch.tensor(ops, dtype=torch.uint8, device="cuda"),
            torch.tensor(np.array(ex, dtype=np.uint64).view(np.int64), device="cuda"))


def test_kv_protect_batch(gpu, oracle, golden):
    import speedb_amd as S
    torch = gpu
    blob = golden["blob"]
    dev = torch.frombuffer(bytearray(blob + bytes(64)), dtype=torch.uint8).to("cuda")
    for mode in range(4):
        cs = [c for c in golden["kv_protect"] if c["mode"] == mode]
        ks = spans(torch, S, dev, [c["koff"] for c in cs], [c["klen"] for c in cs])
        vs = spans(torch, S, dev, [c["voff"] for c in cs], [c["vlen"] for c in cs])
        ops = torch.tensor([c["op"] for c in cs], dtype=torch.uint8, device="cuda")
        ex = torch.tensor(np.array([c["extra"] for c in cs], dtype=np.uint64).view(np.int64), device="cuda")
        got = u64(S.kv_protect_batch(mode, ks, vs, ops, ex))
        assert got == [c["out"] for c in cs], mode
    kh, vh, ko, vo, kl, vl, ops, ex, ks, vs, dops, dex = _kv_batch(torch, S, 500, 3000)
    for mode in range(4):
        got = u64(S.kv_protect_batch(mode, ks, vs, dops, dex))
        for i in range(len(kl)):
            want = oracle.KvProtect(mode, kh[ko[i]:ko[i] + kl[i]], vh[vo[i]:vo[i] + vl[i]], ops[i], ex[i])
            assert got[i] == want, (mode, i, kl[i], vl[i])


def test_kv_protect_key_classes(gpu, oracle):
    """Keys of every length 0..40 (the 0 / 1-3 / 4-8 / 9-16 / 17+ XXPH3
    classes; keys <= 16 bytes are hashed from the two prefetched words) at
    every byte alignment."""
    import speedb_amd as S
    torch = gpu
    klen = [n for n in range(41) for _ in range(8)]
    vlen = [(37 * i) % 1500 for i in range(len(klen))]
    kh, kd, ko, _ = make_batch(torch, 77, klen)
    vh, vd, vo, _ = make_batch(torch, 78, vlen)
    ops = [(5 * i) % 256 for i in range(len(klen))]
    ex = [(0x9E3779B97F4A7C15 * (i + 1)) & (2 ** 64 - 1) for i in range(len(klen))]
    ks, vs = spans(torch, S, kd, ko, klen), spans(torch, S, vd, vo, vlen)
    dops = torch.tensor(ops, dtype=torch.uint8, device="cuda")
    dex = torch.tensor(np.array(ex, dtype=np.uint64).view(np.int64), device="cuda")
    for mode in range(4):
        got = u64(S.kv_protect_batch(mode, ks, vs, dops, dex))
        for i in range(len(klen)):
            want = oracle.KvProtect(mode, kh[ko[i]:ko[i] + klen[i]], vh[vo[i]:vo[i] + vlen[i]], ops[i], ex[i])
            assert got[i] == want, (mode, i, klen[i], vlen[i])


@pytest.mark.parametrize("prot_bytes", [1, 2, 4, 8])
def test_kv_protect_verify(gpu, oracle, prot_bytes):
    """ProtectionInfo::Verify(len, ptr): stored = Encode(len) of the right
    value verifies; one flipped value byte is caught (for 1-byte protection a
    collision is possible, so compare with the oracle's own verdict)."""
    import speedb_amd as S
    torch = gpu
    kh, vh, ko, vo, kl, vl, ops, ex, ks, vs, dops, dex = _kv_batch(torch, S, 900 + prot_bytes, 1000)
    mode = int(S.ProtectionKind.KVOS)
    want = [oracle.KvProtect(mode, kh[ko[i]:ko[i] + kl[i]], vh[vo[i]:vo[i] + vl[i]], ops[i], ex[i])
            for i in range(len(kl))]
    stored = b"".join(struct.pack("<Q", w)[:prot_bytes] for w in want)
    dst = torch.frombuffer(bytearray(stored), dtype=torch.uint8).to("cuda")
    mm, cnt, comp = S.kv_protect_verify_batch(mode, ks, vs, dst, prot_bytes, dops, dex)
    assert int(cnt.item()) == 0 and not bool(mm.any())
    assert u64(comp) == want
    # corrupt one value byte of 20 KVs with non-empty values
    bad = [i for i in random.Random(prot_bytes).sample(range(len(kl)), 60) if vl[i] > 0][:20]
    vbuf = bytearray(vh)
    for i in bad:
        vbuf[vo[i] + vl[i] // 2] ^= 0x40
    vd = torch.frombuffer(bytearray(bytes(vbuf) + bytes(4096)), dtype=torch.uint8).to("cuda")
    vs2 = S.Spans(vd, vs.count, offsets=vs.offsets, lengths=vs.lengths)
    mm, cnt, _ = S.kv_protect_verify_batch(mode, ks, vs2, dst, prot_bytes, dops, dex)
    exp = []
    for i in range(len(kl)):
        w = oracle.KvProtect(mode, kh[ko[i]:ko[i] + kl[i]], bytes(vbuf[vo[i]:vo[i] + vl[i]]), ops[i], ex[i])
        exp.append(int(struct.pack("<Q", w)[:prot_bytes] != struct.pack("<Q", want[i])[:prot_bytes]))
    assert mm.cpu().tolist() == exp
    assert int(cnt.item()) == sum(exp)
    if prot_bytes >= 4:
        assert sorted(i for i, e in enumerate(exp) if e) == sorted(bad)


def test_large_ragged_batches_static_and_dynamic_feeds(gpu, oracle):
    """Ragged batches whose workgroup shares fit one LDS descriptor window
    and shares of several windows (XXH3: 1024 spans per window; the CRC row
    feed's launches split at its cache): oracle-exact results either way."""
    import speedb_amd as S
    torch = gpu
    rnd = random.Random(77)
    for count in (60_000, 450_000):
        lens = [rnd.choice([0, 1, 7, 64, 100, 240, 241, 700, 1023, 1500, rnd.randrange(0, 2000)])
                for _ in range(count)]
        offs, pos = [], 0
        for n in lens:
            pos += rnd.randrange(0, 8)
            offs.append(pos)
            pos += n
        dev = torch.randint(0, 256, (pos + 4096,), dtype=torch.uint8, device="cuda",
                            generator=torch.Generator(device="cuda").manual_seed(count))
        sp = spans(torch, S, dev, offs, lens)
        crc = u32(S.crc32c_batch(sp))
        x3 = u64(S.xxh3_64_batch(sp))
        host = dev.cpu().numpy().tobytes()
        idx = rnd.sample(range(count), 2500) + list(range(50)) + list(range(count - 50, count))
        for i in idx:
            b = host[offs[i]:offs[i] + lens[i]]
            assert crc[i] == oracle.Value(b), (count, i, lens[i])
            assert x3[i] == oracle.XXH3(b), (count, i, lens[i])


def test_xxh3_long_spans_in_pieces(gpu, oracle):
    """k_xxh3_wave splits spans of more than 4 rounds (16 KiB) into pieces
    dealt to different waves, chained through LDS: lengths at every piece
    boundary (1 KiB segments, the lone partial segment, the last stripe), at
    every start alignment, mixed with short and 4 KiB spans, and spans of
    hundreds of pieces."""
    import speedb_amd as S
    torch = gpu
    rnd = random.Random(41)
    lens = []
    for m in (15, 16, 17, 19, 20, 21, 32, 33, 36, 37, 48, 64, 65, 68, 69, 80, 100, 257):
        for d in (-64, -1, 0, 1, 2, 63, 64, 65, 1023):
            lens.append(1024 * m + d)
    lens += [4 << 20, (4 << 20) + 4097, 0, 3, 240, 241, 5000]
    lens += [rnd.randrange(241, 70_000) for _ in range(4000)]
    rnd.shuffle(lens)
    host, dev, offs, lens = make_batch(torch, 41, lens)
    got = u64(S.xxh3_64_batch(spans(torch, S, dev, offs, lens)))
    for i, (o, n) in enumerate(zip(offs, lens)):
        assert got[i] == oracle.XXH3(host[o:o + n]), (i, o, n)


@pytest.mark.parametrize("where", ["front", "middle", "back"])
def test_empty_workgroup_shares(gpu, oracle, where):
    """Batches whose bytes sit almost all in one span: the XXH3 wave driver's
    byte-balanced shares (share_by_bytes) leave most workgroups an EMPTY
    range, and the CRC kernels' count shares give the long span's workgroup
    all the work -- both hashes must still cover every span exactly once."""
    import speedb_amd as S
    torch = gpu
    rnd = random.Random(61)
    small = [rnd.randrange(0, 400) for _ in range(300)]
    big = 8 << 20
    pos = {"front": 0, "middle": 150, "back": 300}[where]
    lens = small[:pos] + [big] + small[pos:]
    host, dev, offs, lens = make_batch(torch, 61, lens)
    sp = spans(torch, S, dev, offs, lens)
    got_x = u64(S.xxh3_64_batch(sp))
    got_c = u32(S.crc32c_batch(sp))
    for i, (o, n) in enumerate(zip(offs, lens)):
        assert got_x[i] == oracle.XXH3(host[o:o + n]), ("xxh3", i, o, n)
        assert got_c[i] == oracle.Value(host[o:o + n]), ("crc", i, o, n)


# ---- long spans / whole-file checksum -----------------

LONG_SIZES = [0, 1, 15, 16, 4095, 4096, 65535, 65536, 65537, 131072, 3 * 65536 + 5,
              (1 << 20) + 3, (5 << 20) + 4097]


def test_crc32c_long_vs_oracle(gpu, oracle):
    """mck_crc32c_long == crc32c::Extend over the whole span, at piece-boundary
    sizes, every start alignment and random init values."""
    import speedb_amd as S
    torch = gpu
    host = splitmix_bytes(77, (6 << 20) + 256)
    dev = torch.frombuffer(bytearray(host), dtype=torch.uint8).to("cuda")
    rnd = random.Random(78)
    for n in LONG_SIZES:
        for off in (0, 1, 7, 16, 63):
            init = rnd.choice([0, 0xFFFFFFFF, rnd.getrandbits(32)])
            got = int(S.crc32c_long(dev, n, init, offset=off).cpu().numpy().view(np.uint32)[0])
            assert got == oracle.Extend(init, host[off:off + n]), (n, off, init)


def test_file_checksum_generator(gpu, oracle):
    """FileChecksumGenCrc32c (util/file_checksum_helper.h:22-72): the same
    big-endian checksum whether the file arrives as host Updates of any
    cut, or as device-resident regions (UpdateDevice)."""
    import speedb_amd as S
    torch = gpu
    data = splitmix_bytes(4546, (3 << 20) + 17)
    want = oracle.FileChecksumCrc32c(data)
    fac = S.GetFileChecksumGenCrc32cFactory()
    assert fac.Name() == "FileChecksumGenCrc32cFactory"
    assert fac.CreateFileChecksumGenerator(S.FileChecksumGenContext("f", "Other")) is None
    g_host = fac.CreateFileChecksumGenerator(S.FileChecksumGenContext("f", ""))
    g_dev = fac.CreateFileChecksumGenerator(S.FileChecksumGenContext("f", "FileChecksumCrc32c"))
    pos, step = 0, 1
    while pos < len(data):
        g_host.Update(data[pos:pos + step])
        pos += step
        step = step * 5 + 1
    dev = torch.frombuffer(bytearray(data + bytes(64)), dtype=torch.uint8).to("cuda")
    cuts = [0, 3, 70000, (1 << 20) + 9, len(data)]
    for a, b in zip(cuts, cuts[1:]):
        g_dev.UpdateDevice(dev, b - a, offset=a)
    for g in (g_host, g_dev):
        g.Finalize()
        assert g.GetChecksum() == want
        assert g.Name() == S.kStandardDbFileChecksumFuncName
    g0 = S.FileChecksumGenCrc32c()
    g0.Update(b"123456789")  # util/crc32c_test.cc:81
    g0.Finalize()
    assert g0.GetChecksum() == bytes.fromhex("e3069283")


def test_crc32c_long_full_size_combine(gpu, oracle):
    """At full size (1 GiB + odd tail) the long-span CRC equals the host
    Crc32cCombine fold of the uniform batch kernel's per-4 KiB CRCs -- two
    device paths and the host algebra agree (a size-independent property)."""
    import speedb_amd as S
    torch = gpu
    n_blocks, tail = 1 << 18, 12345
    g = torch.Generator(device="cuda")
    g.manual_seed(9)
    dev = torch.randint(0, 256, (n_blocks * 4096 + tail + 64,), dtype=torch.uint8, device="cuda",
                        generator=g)
    per = S.crc32c_batch(S.Spans.uniform(dev, 4096, n_blocks)).cpu().numpy().view(np.uint32)
    tail_crc = int(S.crc32c_batch(S.Spans(dev[n_blocks * 4096:], 1, stride=0, length=tail))
                   .cpu().numpy().view(np.uint32)[0])
    acc = 0
    for v in per.tolist():
        acc = oracle.Combine(acc, int(v), 4096)
    acc = oracle.Combine(acc, tail_crc, tail)
    got = int(S.crc32c_long(dev, n_blocks * 4096 + tail).cpu().numpy().view(np.uint32)[0])
    assert got == acc


@pytest.mark.parametrize("ctype", [1, 4])
def test_sst_verify_large_static_feed(gpu, oracle, ctype):
    """More blocks than the per-workgroup LDS descriptor caches (the static
    feeds of the CRC and XXH3 drivers, whose first span per wave has a
    wave-uniform address): small blocks at odd offsets, trailers computed on
    the device and checked against the oracle on a sample that includes the
    first blocks of every wave, then one flipped byte per corrupted block."""
    import speedb_amd as S
    torch = gpu
    n = 420_000
    rng = np.random.default_rng(ctype)
    lens = rng.integers(50, 300, n)
    offs = np.concatenate([[3], 3 + np.cumsum(lens + 5)[:-1]])
    total = int(offs[-1] + lens[-1] + 5)
    host = bytearray(rng.integers(0, 256, total + 64, dtype=np.uint8).tobytes())
    comps = rng.integers(0, 2, n).astype(np.uint8)
    dev = torch.frombuffer(bytes(host), dtype=torch.uint8).to("cuda")
    sp = spans(torch, S, dev, offs.tolist(), lens.tolist())
    ct = torch.tensor(comps, device="cuda")
    tr = np.array(u32(S.sst_trailer_batch(ctype, sp, ct)), dtype=np.uint32)
    for i in list(range(0, 5000)) + list(range(5000, n, 211)) + [n - 1]:
        o, ln = int(offs[i]), int(lens[i])
        assert tr[i] == oracle.BuiltinLast(ctype, bytes(host[o:o + ln]), int(comps[i])), i
    arr = np.frombuffer(host, dtype=np.uint8).copy()
    arr[offs + lens] = comps
    trb = tr.view(np.uint8).reshape(n, 4)
    for k in range(4):
        arr[offs + lens + 1 + k] = trb[:, k]
    bad = sorted(set([0, 1, 17, 4095, 4096, 9000] + rng.integers(0, n, 20).tolist()))
    for i in bad:
        arr[offs[i] + rng.integers(0, lens[i])] ^= 0x10
    dev2 = torch.from_numpy(arr).to("cuda")
    sp2 = spans(torch, S, dev2, offs.tolist(), lens.tolist())
    mm, comp, stored, cnt = S.sst_verify_batch(ctype, sp2)
    flagged = np.nonzero(mm.cpu().numpy())[0].tolist()
    assert flagged == bad
    assert int(cnt.item()) == len(bad)

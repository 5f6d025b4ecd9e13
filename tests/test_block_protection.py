"""Per-KV protection of block entries:
table/block_based/block.cc:1091-1222 Block::Initialize{Data,Index,MetaIndex}
BlockProtectionInfo, block.h:271-274 GenerateKVChecksum, block.h:567-574
PerKVChecksumCorruptionError.

Blocks come from the BlockBuilder restatement in tests/sst_format.py (the
reference's block.cc cannot be built here: it needs util/comparator.cc and
db/dbformat.cc, which pull in the options/Customizable framework and the
arena -- so the entry layout is "parity unpinned", as for the SST files).
Each block's expected kv_checksum array is computed two ways: entry by entry
from the writer's (key, value) list with ProtectKV (oracle, pinned to the
reference's db/kv_checksum.h through oracle/_ref), and by the oracle's walk
of the encoded block; the GPU must match both byte for byte.
"""
import random
import struct

import pytest

from sst_format import build_block, common_prefix, handle, varint, varsigned

DATA, INDEX, INDEX_DELTA, INDEX_DELTA_FK, META = 0, 1, 2, 3, 4
OK, BAD_CONTENTS, BAD_ENTRY, BAD_RESTARTS = 0, 1, 2, 3


def sorted_keys(rnd, n, klo=8, khi=40, prefix=b"", internal=True):
    """n distinct sorted keys sharing prefixes (user key [+ 8-byte seq/type
    footer, as internal keys in data blocks])."""
    ks = set()
    while len(ks) < n:
        k = prefix + b"k%06d" % rnd.randrange(10 * n + 10)
        k += bytes(rnd.getrandbits(8) for _ in range(rnd.randrange(max(0, klo - len(k)), max(1, khi - len(k)))))
        ks.add(k)
    out = sorted(ks)
    if internal:
        out = [k + struct.pack("<Q", (rnd.getrandbits(56) << 8) | rnd.randrange(2)) for k in out]
    return out


def data_block(rnd, n, ri, vlo=0, vhi=300, **kw):
    keys = sorted_keys(rnd, n, **kw)
    entries = [(k, bytes(rnd.getrandbits(8) for _ in range(rnd.randrange(vlo, vhi + 1)))) for k in keys]
    return entries


def raw_kvs(entries, ri, deltas=None):
    """(key, raw value) per entry as the iterator sees them (block_builder.cc
    :188-252: delta value only when shared != 0)."""
    out, last = [], b""
    for i, (k, v) in enumerate(entries):
        shared = 0 if i % ri == 0 else common_prefix(last, k)
        raw = v if deltas is None or shared == 0 else deltas[i]
        out.append((k, raw))
        last = k
    return out


def index_entries(rnd, n, first_key):
    keys = sorted_keys(rnd, n, 6, 30, internal=False)
    handles, off = [], rnd.randrange(1 << 20)
    for _ in range(n):
        sz = rnd.randrange(100, 70000)
        handles.append((off, sz))
        off += sz + 5
    entries, deltas, prev = [], [], None
    for i, (k, h) in enumerate(zip(keys, handles)):
        v = handle(*h)
        dv = varsigned(h[1] - prev[1]) if prev is not None else b""
        if first_key:
            fk = varint(len(k) + 3) + k + b"fk!"
            v += fk
            dv += fk
        entries.append((k, v))
        deltas.append(dv)
        prev = h
    return entries, deltas


def expected(oracle, kvs, p):
    out = bytearray()
    for k, v in kvs:
        out += struct.pack("<Q", oracle.KvProtect(0, k, v))[:p]
    return bytes(out)


def corpus(rnd):
    """(kind, block bytes, expected kv_checksum or None, expected status)."""
    cases = []
    for ri in (1, 2, 3, 16, 64):
        for n in (1, 5, 16, 17, 100):
            e = data_block(rnd, n, ri)
            cases.append((DATA, build_block(e, ri), raw_kvs(e, ri), OK))
    # > 64 restart intervals (lane chunk loop), long keys / values (XXPH3 long path)
    e = data_block(rnd, 300, 2, 0, 40)
    cases.append((DATA, build_block(e, 2), raw_kvs(e, 2), OK))
    e = data_block(rnd, 20, 4, 200, 3000, klo=100, khi=400)
    cases.append((DATA, build_block(e, 4), raw_kvs(e, 4), OK))
    # hash-index footers (kDataBlockBinaryAndHash)
    for nb in (1, 7, 200):
        e = data_block(rnd, 40, 8)
        cases.append((DATA, build_block(e, 8, hash_buckets=nb), raw_kvs(e, 8), OK))
    # meta index / properties (MetaBlockIter: restart interval 1, no sharing)
    e = sorted((b"rocksdb.%s" % bytes(rnd.choice(b"abcdefgh") for _ in range(rnd.randrange(3, 30))),
                bytes(rnd.getrandbits(8) for _ in range(rnd.randrange(0, 20)))) for _ in range(12))
    e = list(dict(e).items())
    cases.append((META, build_block(e, 1), raw_kvs(e, 1), OK))
    # index blocks: value_is_full, delta-encoded, delta + first key
    for ri in (1, 4, 16):
        e, d = index_entries(rnd, 50, False)
        cases.append((INDEX, build_block(e, ri), raw_kvs(e, ri), OK))
        cases.append((INDEX_DELTA, build_block(e, ri, d), raw_kvs(e, ri, d), OK))
        e, d = index_entries(rnd, 50, True)
        cases.append((INDEX_DELTA_FK, build_block(e, ri, d), raw_kvs(e, ri, d), OK))
    # empty blocks: BlockBuilder's (one restart at 0), and num_restarts == 0
    cases.append((DATA, build_block([], 16), [], OK))
    cases.append((DATA, struct.pack("<I", 0), [], OK))
    # constructor error markers
    cases.append((DATA, b"\x01\x00", None, BAD_CONTENTS))                      # < 4 bytes
    cases.append((DATA, struct.pack("<I", 5), None, BAD_CONTENTS))           # restarts wrap
    good = build_block(data_block(rnd, 30, 4), 4)
    cases.append((DATA, good[:-4] + struct.pack("<I", 10 ** 6), None, BAD_CONTENTS))
    # bad entries: truncated varint, value running into the restart array
    e = data_block(rnd, 10, 4)
    b = bytearray(build_block(e, 4))
    b[2] = 0xFF  # value length of entry 0 now points past the entry area
    cases.append((DATA, bytes(b), None, BAD_ENTRY))
    b = bytearray(build_block(e, 4))
    b[0] = 0x80  # shared varint continues: decodes garbage
    cases.append((DATA, bytes(b), None, None))
    b = bytearray(build_block(e, 4))
    b[0] = 3  # shared != 0 on the block's first entry
    cases.append((DATA, bytes(b), None, BAD_ENTRY))
    # restart layouts BlockBuilder never writes
    e = data_block(rnd, 12, 4)
    blk = build_block(e, 4)
    nr = struct.unpack_from("<I", blk, len(blk) - 4)[0]
    ro = len(blk) - 4 - 4 * nr
    r = list(struct.unpack_from("<%dI" % nr, blk, ro))
    r2 = [r[0], r[2], r[1]]
    cases.append((DATA, blk[:ro] + struct.pack("<3I", *r2) + blk[-4:], None, BAD_RESTARTS))
    r2 = [r[0], r[1] + 1, r[2]]  # restart inside an entry
    cases.append((DATA, blk[:ro] + struct.pack("<3I", *r2) + blk[-4:], None, BAD_RESTARTS))
    e2 = data_block(rnd, 7, 3)
    # hand-made block: restarts at entries 0, 2, 5 of a 7-entry run (2, 3, 2)
    body, restarts, last = bytearray(), [], b""
    for i, (k, v) in enumerate(e2):
        if i in (0, 2, 5):
            restarts.append(len(body))
            sh = 0
        else:
            sh = common_prefix(last, k)
        body += varint(sh) + varint(len(k) - sh) + varint(len(v)) + k[sh:] + v
        last = k
    blk = bytes(body) + struct.pack("<%dI" % len(restarts), *restarts) + struct.pack("<I", len(restarts))
    cases.append((DATA, blk, None, BAD_RESTARTS))
    return cases


def test_oracle_block_protection(oracle):
    """The oracle's block walk equals ProtectKV over the writer's entries."""
    rnd = random.Random(7)
    for kind, blk, kvs, st in corpus(rnd):
        for p in (1, 8):
            got_st, got, _ = oracle.BlockKvProtect(kind, blk, p)
            if st is not None:
                assert got_st == st, (kind, len(blk), st, got_st)
            if kvs is not None:
                assert got == expected(oracle, kvs, p)


def test_oracle_restart_interval(oracle):
    rnd = random.Random(3)
    for ri, n in ((16, 40), (1, 5), (7, 7), (5, 3)):
        e = data_block(rnd, n, ri)
        st, _, got = oracle.BlockKvProtect(DATA, build_block(e, ri), 4)
        assert st == OK
        # GetRestartInterval (block.h:484-497): 0 with a single restart
        assert got == (0 if (n + ri - 1) // ri <= 1 else ri)


def test_ref_pins_protect_kv(oracle, ref):
    """The per-entry function is the reference's own ProtectKV (_ref build of
    db/kv_checksum.h)."""
    if ref is None:
        pytest.skip("oracle/_ref not built")
    rnd = random.Random(11)
    for kind, blk, kvs, st in corpus(rnd)[:40]:
        for k, v in (kvs or []):
            assert oracle.KvProtect(0, k, v) == ref.ref_kv_protect(0, k, len(k), v, len(v), 0, 0)


# ---------------------------------------------------------------------------
# GPU parity
# ---------------------------------------------------------------------------


def _pack(torch, blocks, rnd, align_any=True):
    """Blocks at byte offsets in one device buffer (odd offsets: blocks sit
    after 5-byte trailers in an SST)."""
    offs, buf = [], bytearray()
    for b in blocks:
        buf += bytes(rnd.randrange(0, 7) if align_any else 0)
        offs.append(len(buf))
        buf += b
    buf += bytes(64)
    dev = torch.frombuffer(bytearray(buf), dtype=torch.uint8).to("cuda")
    return dev, torch.tensor(offs, dtype=torch.int64, device="cuda"), \
        torch.tensor([len(b) for b in blocks], dtype=torch.int32, device="cuda")


@pytest.mark.gpu
def test_block_protection_gpu_vs_oracle(gpu, oracle):
    import speedb_amd
    from speedb_amd import block as B
    torch = gpu
    rnd = random.Random(21)
    cases = corpus(rnd)
    for kind in (DATA, INDEX, INDEX_DELTA, INDEX_DELTA_FK, META):
        sel = [c for c in cases if c[0] == kind or (kind == DATA and c[0] not in (INDEX, INDEX_DELTA,
                                                                                   INDEX_DELTA_FK, META))]
        blocks = [c[1] for c in sel]
        base, offs, lens = _pack(torch, blocks, rnd)
        spans = speedb_amd.Spans(base, len(blocks), offs, lens)
        for p in (1, 2, 4, 8):
            prot = B.InitializeBlockProtectionInfo(kind, spans, p)
            torch.cuda.synchronize()
            kb = prot.key_base.cpu().tolist()
            sts = prot.status.cpu().tolist()
            ris = prot.restart_interval.cpu().tolist()
            allck = prot.kv_checksum.cpu().numpy().tobytes()
            for i, blk in enumerate(blocks):
                ost, ock, ori = oracle.BlockKvProtect(kind, blk, p)
                assert sts[i] == ost, (kind, i, sts[i], ost)
                assert allck[kb[i] * p:kb[i + 1] * p] == ock, (kind, i)
                assert ris[i] == ori, (kind, i)


@pytest.mark.gpu
def test_block_protection_verify_flags_exact_entries(gpu, oracle):
    import speedb_amd
    from speedb_amd import block as B
    torch = gpu
    rnd = random.Random(5)
    blocks = [build_block(data_block(rnd, rnd.randrange(1, 60), rnd.choice((1, 4, 16))), 16) for _ in range(300)]
    base, offs, lens = _pack(torch, blocks, rnd)
    spans = speedb_amd.Spans(base, len(blocks), offs, lens)
    prot = B.InitializeDataBlockProtectionInfo(spans, 2)
    mism, cnt = B.VerifyBlockProtectionInfo(spans, prot)
    assert int(cnt.item()) == 0 and int(mism.sum().item()) == 0
    stored = prot.kv_checksum.clone()
    bad = sorted(rnd.sample(range(prot.total_keys), 25))
    for k in bad:
        stored[2 * k + rnd.randrange(2)] ^= 1 << rnd.randrange(8)
    mism, cnt = B.VerifyBlockProtectionInfo(spans, prot, stored)
    assert int(cnt.item()) == len(bad)
    assert torch.nonzero(mism).flatten().cpu().tolist() == bad
    st = B.PerKVChecksumStatus(prot, mism)
    assert st and st[0][1].IsCorruption() and "per key-value checksum verification failed" in st[0][1].message


@pytest.mark.gpu
@pytest.mark.parametrize("p", [1, 8])
def test_block_protection_long_value_list(gpu, oracle, p):
    """Values over 240 bytes go through the long-value list (k_block_kv_t
    records them by key index, k_block_long hashes them in key order): blocks
    of 241..3000-byte values mixed with short ones, protect against the
    oracle, then verify with corrupted stored bytes on long and short
    entries alike."""
    import speedb_amd
    from speedb_amd import block as B
    torch = gpu
    rnd = random.Random(70 + p)
    blocks = [build_block(data_block(rnd, rnd.randrange(1, 12), rnd.choice((1, 2, 16)),
                                     rnd.choice((0, 241, 241)), rnd.choice((300, 1100, 3000))), 16)
              for _ in range(400)]
    base, offs, lens = _pack(torch, blocks, rnd)
    spans = speedb_amd.Spans(base, len(blocks), offs, lens)
    prot = B.InitializeDataBlockProtectionInfo(spans, p)
    kb = prot.key_base.cpu().tolist()
    ck = prot.kv_checksum.cpu().numpy().tobytes()
    for i, blk in enumerate(blocks):
        assert ck[kb[i] * p:kb[i + 1] * p] == oracle.BlockKvProtect(DATA, blk, p)[1], i
    mism, cnt = B.VerifyBlockProtectionInfo(spans, prot)
    assert int(cnt.item()) == 0 and int(mism.sum().item()) == 0
    stored = prot.kv_checksum.clone()
    bad = sorted(rnd.sample(range(prot.total_keys), 40))
    for k in bad:
        stored[p * k + rnd.randrange(p)] ^= 1 << rnd.randrange(8)
    mism, cnt = B.VerifyBlockProtectionInfo(spans, prot, stored)
    assert int(cnt.item()) == len(bad)
    assert torch.nonzero(mism).flatten().cpu().tolist() == bad


@pytest.mark.gpu
def test_block_protection_many_blocks_property(gpu, oracle):
    """> 2048 blocks (multi-tile scans): 64 distinct blocks tiled 80 times --
    every copy's checksums equal its original's (the oracle's)."""
    import speedb_amd
    from speedb_amd import block as B
    torch = gpu
    rnd = random.Random(9)
    uniq = [build_block(data_block(rnd, rnd.randrange(20, 45), 8, 50, 120), 16) for _ in range(64)]
    want = [oracle.BlockKvProtect(DATA, b, 4)[1] for b in uniq]
    blocks = uniq * 80
    base, offs, lens = _pack(torch, blocks, rnd)
    spans = speedb_amd.Spans(base, len(blocks), offs, lens)
    prot = B.InitializeDataBlockProtectionInfo(spans, 4)
    kb = prot.key_base.cpu().tolist()
    ck = prot.kv_checksum.cpu().numpy().tobytes()
    assert prot.total_keys == sum(len(w) // 4 for w in want) * 80
    for i in range(len(blocks)):
        assert ck[kb[i] * 4:kb[i + 1] * 4] == want[i % 64]


@pytest.mark.gpu
def test_block_protection_one_pass_vs_oracle(gpu, oracle):
    """mck_block_kv_protect_blocks_batch (layout checks and hashing in one
    walk, entries parked in per-block slots) with room for every block of the
    corpus -- 300-entry blocks, 100..400-byte keys in the per-block arena --
    equals the oracle block by block (status, checksums, restart interval),
    and its key_base / arena_base equal the two-pass layout's."""
    import speedb_amd
    from speedb_amd import block as B
    torch = gpu
    rnd = random.Random(23)
    cases = corpus(rnd)
    for kind in (DATA, INDEX, INDEX_DELTA, INDEX_DELTA_FK, META):
        sel = [c for c in cases if c[0] == kind or (kind == DATA and c[0] not in (INDEX, INDEX_DELTA,
                                                                                   INDEX_DELTA_FK, META))]
        blocks = [c[1] for c in sel]
        base, offs, lens = _pack(torch, blocks, rnd)
        spans = speedb_amd.Spans(base, len(blocks), offs, lens)
        for p in (1, 2, 4, 8):
            prot = B.InitializeBlockProtectionInfoOnePass(kind, spans, p, slot_cap=320, arena_cap=4096)
            two = B.InitializeBlockProtectionInfo(kind, spans, p, one_pass=False)
            torch.cuda.synchronize()
            kb = prot.key_base.cpu().tolist()
            sts = prot.status.cpu().tolist()
            ris = prot.restart_interval.cpu().tolist()
            allck = prot.kv_checksum.cpu().numpy().tobytes()
            for i, blk in enumerate(blocks):
                ost, ock, ori = oracle.BlockKvProtect(kind, blk, p)
                assert sts[i] == ost, (kind, i, sts[i], ost)
                assert allck[kb[i] * p:kb[i + 1] * p] == ock, (kind, i)
                assert ris[i] == ori, (kind, i)
            assert kb == two.key_base.cpu().tolist()
            assert prot.arena_base.cpu().tolist() == two.arena_base.cpu().tolist()
            assert prot.total_keys == two.total_keys


@pytest.mark.gpu
def test_block_protection_one_pass_overflow(gpu, oracle):
    """Blocks with more entries than slot_cap, or a key over 128 bytes and
    arena_cap, come back MCK_BLOCK_SLOT_OVERFLOW with no keys while their
    neighbours are protected; InitializeBlockProtectionInfo then runs the
    two-pass pair for the batch and matches the oracle everywhere."""
    import speedb_amd
    from speedb_amd import block as B
    torch = gpu
    rnd = random.Random(29)
    small = [build_block(data_block(rnd, rnd.randrange(1, 16), 4), 4) for _ in range(40)]
    big = build_block(data_block(rnd, 40, 4), 4)
    longk = build_block(data_block(rnd, 6, 2, klo=130, khi=200), 2)
    blocks = small[:20] + [big] + small[20:] + [longk]
    base, offs, lens = _pack(torch, blocks, rnd)
    spans = speedb_amd.Spans(base, len(blocks), offs, lens)
    prot = B.InitializeBlockProtectionInfoOnePass(DATA, spans, 8, slot_cap=16, arena_cap=0)
    sts = prot.status.cpu().tolist()
    assert sts[20] == B.BlockStatus.kSlotOverflow and sts[-1] == B.BlockStatus.kSlotOverflow
    kb = prot.key_base.cpu().tolist()
    ck = prot.kv_checksum.cpu().numpy().tobytes()
    for i, blk in enumerate(blocks):
        if i in (20, len(blocks) - 1):
            assert kb[i + 1] == kb[i]
            continue
        assert sts[i] == OK
        assert ck[kb[i] * 8:kb[i + 1] * 8] == oracle.BlockKvProtect(DATA, blk, 8)[1], i
    # the long key fits once the arena slice holds it
    prot = B.InitializeBlockProtectionInfoOnePass(DATA, spans, 8, slot_cap=64, arena_cap=256)
    assert prot.status.cpu().tolist() == [OK] * len(blocks)
    full = B.InitializeDataBlockProtectionInfo(spans, 8)
    kb = full.key_base.cpu().tolist()
    ck = full.kv_checksum.cpu().numpy().tobytes()
    assert full.slot_cap == 0  # the fallback ran
    for i, blk in enumerate(blocks):
        assert ck[kb[i] * 8:kb[i + 1] * 8] == oracle.BlockKvProtect(DATA, blk, 8)[1], i


@pytest.mark.gpu
def test_block_protection_one_pass_equals_two_pass_many(gpu):
    """Property at scale: 3000 blocks (short and long values, long keys,
    corrupt blocks, every 7th block 64 bytes of garbage) -- the one-pass
    entry point (room for every block) and the two-pass pair agree on every
    status, restart interval, key base and checksum byte, and one-pass
    verify flags exactly the entries whose stored bytes were flipped."""
    import speedb_amd
    from speedb_amd import block as B
    torch = gpu
    rnd = random.Random(41)
    blocks = []
    for i in range(3000):
        if i % 7 == 3:
            blocks.append(bytes(rnd.getrandbits(8) for _ in range(64)))
            continue
        n = rnd.randrange(1, 40)
        ri = rnd.choice((1, 2, 4, 16))
        if i % 11 == 5:
            e = data_block(rnd, n, ri, 200, 1500)
        elif i % 13 == 6:
            e = data_block(rnd, rnd.randrange(1, 8), ri, 0, 60, klo=130, khi=300)
        else:
            e = data_block(rnd, n, ri, 0, 130)
        blocks.append(build_block(e, ri))
    base, offs, lens = _pack(torch, blocks, rnd)
    spans = speedb_amd.Spans(base, len(blocks), offs, lens)
    for p in (2, 8):
        one = B.InitializeBlockProtectionInfoOnePass(DATA, spans, p, slot_cap=64, arena_cap=512)
        two = B.InitializeBlockProtectionInfo(DATA, spans, p, one_pass=False)
        assert one.status.cpu().tolist() == two.status.cpu().tolist()
        assert one.restart_interval.cpu().tolist() == two.restart_interval.cpu().tolist()
        assert one.key_base.cpu().tolist() == two.key_base.cpu().tolist()
        assert one.arena_base.cpu().tolist() == two.arena_base.cpu().tolist()
        assert torch.equal(one.kv_checksum, two.kv_checksum)
        stored = one.kv_checksum.clone()
        bad = sorted(rnd.sample(range(one.total_keys), 50))
        for k in bad:
            stored[p * k + rnd.randrange(p)] ^= 1 << rnd.randrange(8)
        mism, cnt = B.VerifyBlockProtectionInfo(spans, one, stored)
        assert int(cnt.item()) == len(bad)
        assert torch.nonzero(mism).flatten().cpu().tolist() == bad


@pytest.mark.gpu
@pytest.mark.parametrize("count", [1, 63, 64, 65, 129, 200])
def test_block_protection_one_pass_chunk_edges(gpu, count):
    """The one-pass walk keeps its slots interleaved by wave (entry e of a
    wave's 64 blocks side by side, blk_slot_at) and the flush takes a
    workgroup per 64-block chunk: batches of 1 block, around one and two
    chunks, and a ragged last chunk agree with the two-pass pair on every
    status, key base and checksum byte (blocks of 1..40 entries, restart
    intervals 1..16, so walks end at different iterations)."""
    import speedb_amd
    from speedb_amd import block as B
    torch = gpu
    rnd = random.Random(count)
    blocks = []
    for i in range(count):
        ri = rnd.choice((1, 3, 16))
        blocks.append(build_block(data_block(rnd, rnd.randrange(1, 41), ri, 0, 130 if i % 5 else 400), ri))
    base, offs, lens = _pack(torch, blocks, rnd)
    spans = speedb_amd.Spans(base, len(blocks), offs, lens)
    for p in (1, 8):
        one = B.InitializeBlockProtectionInfoOnePass(DATA, spans, p, slot_cap=64, arena_cap=512)
        two = B.InitializeBlockProtectionInfo(DATA, spans, p, one_pass=False)
        assert one.status.cpu().tolist() == two.status.cpu().tolist()
        assert one.key_base.cpu().tolist() == two.key_base.cpu().tolist()
        assert torch.equal(one.kv_checksum, two.kv_checksum)
        mism, cnt = B.VerifyBlockProtectionInfo(spans, one, one.kv_checksum.clone())
        assert int(cnt.item()) == 0


def _corrupt_cases(rnd, blocks):
    """Block-data corruptions: (block index, new bytes, whole)
    -- whole: the block no longer walks to its protect-time entry count, so
    every one of its keys must be flagged."""
    out = []
    mid, last = len(blocks) // 2, len(blocks) - 1
    # num_restarts far past the block: the constructor's error marker
    b = bytearray(blocks[mid])
    b[-4:] = struct.pack("<I", 0x7000)
    out.append((mid, bytes(b), True))
    # shared != 0 at the first entry (a restart point)
    b = bytearray(blocks[last])
    b[0] = 3
    out.append((last, bytes(b), True))
    # a restart offset moved into the middle of an entry (one-pass walk:
    # bad restarts; either way the key count or layout changes)
    b = bytearray(blocks[mid + 1])
    nr = struct.unpack("<I", b[-4:])[0]
    if nr > 1:
        ro = len(b) - 4 * (nr + 1)
        r1 = struct.unpack("<I", b[ro + 4:ro + 8])[0]
        b[ro + 4:ro + 8] = struct.pack("<I", r1 + 1)
        out.append((mid + 1, bytes(b), None))
    # a value byte of entry 0 (blocks[3] is built with restart interval 1
    # and one-byte varints: its value starts at 3 + key length): only that
    # entry's checksum changes
    b = bytearray(blocks[3])
    b[3 + b[1]] ^= 0x40
    out.append((3, bytes(b), False))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("p", [2, 8])
def test_block_protection_verify_corrupt_block_data(gpu, p):
    """Verify after the BLOCK DATA changed (not only the stored bytes): a
    corrupt header, a bad first entry or a moved restart point in a middle
    block and in the last block.  Both verify entry points index `stored` by
    the protect-time key_base (block.h:623); a block that no longer walks to
    its protect-time entry count has all of its keys flagged, and no key of
    another block is -- the one-pass walk used to re-derive key_base and shift
    every later block (and read `stored` past its end).  The C calls run with
    4 KiB guard bands around `stored` and `mismatch`."""
    import ctypes
    import speedb_amd
    from speedb_amd import block as B
    from speedb_amd._lib import lib
    torch = gpu
    rnd = random.Random(91 + p)
    blocks = []
    for i in range(200):
        n = rnd.randrange(8, 40)
        ri = rnd.choice((2, 4, 16))
        e = data_block(rnd, n, ri, 200, 700) if i % 9 == 4 else data_block(rnd, n, ri, 0, 120)
        blocks.append(build_block(e, ri))
    blocks[3] = build_block(data_block(rnd, 10, 1, 5, 100), 1)
    for idx, nb, whole in _corrupt_cases(rnd, blocks):
        good_base, offs, lens = _pack(torch, blocks, random.Random(1))
        spans = speedb_amd.Spans(good_base, len(blocks), offs, lens)
        for one_pass in (True, False):
            prot = B.InitializeBlockProtectionInfo(DATA, spans, p, one_pass=one_pass)
            assert prot.status.cpu().tolist() == [OK] * len(blocks)
            kb = prot.key_base.cpu().tolist()
            bad_blocks = list(blocks)
            bad_blocks[idx] = nb
            base2, offs2, lens2 = _pack(torch, bad_blocks, random.Random(1))
            assert torch.equal(offs2, offs) and torch.equal(lens2, lens)
            spans2 = speedb_amd.Spans(base2, len(blocks), offs2, lens2)
            mism, cnt, st = B.VerifyBlockProtectionInfo(spans2, prot, return_status=True)
            flagged = torch.nonzero(mism).flatten().cpu().tolist()
            own = list(range(kb[idx], kb[idx + 1]))
            assert set(flagged) <= set(own), (idx, one_pass)
            assert int(cnt.item()) == len(flagged)
            w = whole
            if w is None:  # a moved restart point: the sequential two-pass walk never reads it
                w = True if one_pass else None
            if w is not None:
                assert flagged
            if w is True:
                assert flagged == own
            elif w is False:
                assert flagged == [kb[idx]]
            if one_pass and w:
                assert st is not None and int(st[idx].item()) != OK
                msgs = B.PerKVChecksumStatus(prot, mism, status=st)
                assert [m[0] for m in msgs] == [idx] and "per key-value" not in msgs[0][1].message
            # the C entry points with guard bands around stored / mismatch
            G = 4096
            K = prot.total_keys
            sbuf = torch.full((G + K * p + G,), 0xA5, dtype=torch.uint8, device="cuda")
            sbuf[G:G + K * p] = prot.kv_checksum
            mbuf = torch.full((G + K + G,), 0x5A, dtype=torch.uint8, device="cuda")
            c32 = torch.zeros(1, dtype=torch.int32, device="cuda")
            s = spans2.c()
            if one_pass:
                n = len(blocks)
                status = torch.empty(n, dtype=torch.int32, device="cuda")
                ri = torch.empty(n, dtype=torch.int32, device="cuda")
                work = torch.empty(int(lib.mck_block_kv_blocks_work_bytes(n, prot.slot_cap, prot.arena_cap)),
                                   dtype=torch.uint8, device="cuda")
                rc = lib.mck_block_kv_verify_blocks_batch(
                    DATA, ctypes.byref(s), p, prot.slot_cap, prot.arena_cap, prot.key_base.data_ptr(), K,
                    ri.data_ptr(), status.data_ptr(), work.data_ptr(), sbuf[G:].data_ptr(), mbuf[G:].data_ptr(),
                    c32.data_ptr(), None)
            else:
                work = torch.empty(int(lib.mck_block_kv_work_bytes(K, prot.total_key_bytes)), dtype=torch.uint8,
                                   device="cuda")
                rc = lib.mck_block_kv_verify_batch(
                    DATA, ctypes.byref(s), p, prot.key_base.data_ptr(), prot.arena_base.data_ptr(),
                    prot.restart_interval.data_ptr(), K, work.data_ptr(), sbuf[G:].data_ptr(),
                    mbuf[G:].data_ptr(), c32.data_ptr(), None)
            assert rc == 0
            torch.cuda.synchronize()
            assert bool((sbuf[:G] == 0xA5).all()) and bool((sbuf[G + K * p:] == 0xA5).all())
            assert bool((mbuf[:G] == 0x5A).all()) and bool((mbuf[G + K:] == 0x5A).all())
            assert torch.nonzero(mbuf[G:G + K]).flatten().cpu().tolist() == flagged
            assert int(c32.item()) == len(flagged)


@pytest.mark.gpu
def test_block_protection_verify_overflow_fallback_keeps_walk(gpu):
    """a block that outgrows the one-pass slots at VERIFY time
    sends the batch's entries to the two-pass verify.  A neighbour whose
    restart point moved must still have all of its keys flagged and its
    layout status returned -- the verdict of one block does not depend on
    whether another block of the batch overflowed."""
    import speedb_amd
    from speedb_amd import block as B
    torch = gpu
    rnd = random.Random(77)
    blocks = [build_block(data_block(rnd, rnd.randrange(8, 30), 4, 0, 60), 4) for _ in range(40)]
    grow, moved = 7, 21
    base, offs, lens = _pack(torch, blocks, random.Random(3))
    spans = speedb_amd.Spans(base, len(blocks), offs, lens)
    prot = B.InitializeBlockProtectionInfoOnePass(DATA, spans, 8, slot_cap=32, arena_cap=512)
    assert prot.status.cpu().tolist() == [OK] * len(blocks)
    kb = prot.key_base.cpu().tolist()
    bad = list(blocks)
    bad[grow] = build_block(data_block(rnd, 90, 4, 0, 60), 4)  # 90 entries > slot_cap
    b = bytearray(blocks[moved])
    nr = struct.unpack("<I", b[-4:])[0]
    assert nr > 1
    ro = len(b) - 4 * (nr + 1)
    r1 = struct.unpack("<I", b[ro + 4:ro + 8])[0]
    b[ro + 4:ro + 8] = struct.pack("<I", r1 + 1)
    bad[moved] = bytes(b)
    base2, offs2, lens2 = _pack(torch, bad, random.Random(3))
    spans2 = speedb_amd.Spans(base2, len(bad), offs2, lens2)
    mism, cnt, st = B.VerifyBlockProtectionInfo(spans2, prot, return_status=True)
    assert st is not None
    sts = st.cpu().tolist()
    assert sts[grow] == B.BlockStatus.kSlotOverflow
    assert sts[moved] not in (OK, B.BlockStatus.kSlotOverflow)
    flagged = set(torch.nonzero(mism).flatten().cpu().tolist())
    assert set(range(kb[moved], kb[moved + 1])) <= flagged
    assert flagged <= set(range(kb[moved], kb[moved + 1])) | set(range(kb[grow], kb[grow + 1]))
    assert int(cnt.item()) == len(flagged)
    msgs = dict(B.PerKVChecksumStatus(prot, mism, status=st))
    assert moved in msgs and "per key-value" not in msgs[moved].message


@pytest.mark.gpu
def test_block_protection_empty_and_all_bad(gpu):
    import speedb_amd
    from speedb_amd import block as B
    torch = gpu
    base = torch.zeros(64, dtype=torch.uint8, device="cuda")
    prot = B.InitializeDataBlockProtectionInfo(speedb_amd.Spans(base, 0), 8)
    assert prot.total_keys == 0
    offs = torch.tensor([0, 8], dtype=torch.int64, device="cuda")
    lens = torch.tensor([2, 3], dtype=torch.int32, device="cuda")
    prot = B.InitializeDataBlockProtectionInfo(speedb_amd.Spans(base, 2, offs, lens), 8)
    assert prot.total_keys == 0 and prot.status.cpu().tolist() == [BAD_CONTENTS, BAD_CONTENTS]
    assert not prot.block_status(0).ok() and prot.block_status(0).message == "bad block contents"


def test_block_protection_abi_errors():
    """Argument checks need no GPU."""
    from speedb_amd._lib import lib, mck_spans
    import ctypes
    s = mck_spans(None, None, None, 0, 0, 0)
    assert lib.mck_block_kv_protect_batch(0, ctypes.byref(s), 3, None, None, None, 0, None, None, None) == -1
    assert lib.mck_block_kv_protect_batch(9, ctypes.byref(s), 4, None, None, None, 0, None, None, None) == -1
    assert lib.mck_block_kv_scratch_bytes(5000) >= 16 * 3
    assert lib.mck_block_kv_work_bytes(10, 100) >= 10 * 24 + 100
    assert lib.mck_block_kv_protect_blocks_batch(0, ctypes.byref(s), 3, 64, 0, None, None, None, None, None,
                                                 None, None) == -1
    assert lib.mck_block_kv_protect_blocks_batch(9, ctypes.byref(s), 8, 64, 0, None, None, None, None, None,
                                                 None, None) == -1
    assert lib.mck_block_kv_verify_blocks_batch(0, ctypes.byref(s), 8, 64, 0, None, 0, None, None, None,
                                                None, None, None, None) == -1
    assert lib.mck_block_kv_blocks_work_bytes(10, 64, 32) >= 10 * 64 * 36 + 10 * 32


@pytest.mark.gpu
def test_wave_xxph3_long_loop(gpu, oracle):
    """The block kernels' cooperative XXPH3 long loops -- wave (8
    accumulators x 8 stripe groups), per lane, LDS-staged wave, and four
    spans of different lengths on the four 16-lane rows -- against Hash64
    (mck_internal_xp_wave, an internal test hook)."""
    import ctypes
    from speedb_amd._lib import lib
    torch = gpu
    f = lib.mck_internal_xp_wave
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
    rnd = random.Random(1)
    out = torch.zeros(7, dtype=torch.int64, device="cuda")
    for n in (425, 426, 500, 1000, 1023, 1024, 1025, 1087, 1088, 2100, 5000, 6144):
        b = bytes(rnd.getrandbits(8) for _ in range(n))
        d = torch.frombuffer(bytearray(bytes(rnd.randrange(16)) + b + bytes(64)), dtype=torch.uint8).cuda()
        off = d.numel() - 64 - n
        for seed in (0, 0xD28AAD72F49BD50B):
            assert f(d.data_ptr() + off, n, seed, out.data_ptr(), None) == 0
            r = [x & (2 ** 64 - 1) for x in out.cpu().tolist()]
            want = oracle.Hash64(b, seed)
            assert r[:3] == [want, want, want], (n, seed)
            assert r[3:] == [oracle.Hash64(b[:n - 61 * k], seed) for k in range(4)], (n, seed)

"""Whole-SST-file verification: the engine's host SST
reader (mck_sst_list_blocks) lists exactly the blocks the test-side writer
put into block-based-table images of every footer version / index type, and
the reference's footer errors are reported; on the GPU every block of the
image verifies in one batch and injected corruption is flagged at exactly
the corrupted block (with VerifyBlockChecksum's message)."""
import random
import struct

import pytest

from sst_format import write_sst

CASES = [
    # (format_version, checksum type, index type, delta, meta blocks)
    (0, 1, 0, False, ("filter",)),
    (2, 1, 0, False, ("filter", "range_del")),
    (3, 4, 1, False, ("range_del",)),
    (4, 1, 0, True, ("filter", "compression_dict")),
    (5, 4, 2, True, ("partitioned_filter", "range_del")),
    (5, 1, 3, True, ()),
    (6, 4, 0, True, ("filter", "range_del")),
    (6, 1, 2, True, ("partitioned_filter",)),
    (6, 4, 3, False, ("filter",)),
    (5, 2, 0, True, ("filter",)),   # kxxHash
    (5, 3, 0, True, ()),            # kxxHash64
    (5, 0, 0, True, ("filter",)),   # kNoChecksum
]


def _kinds(blocks):
    return sorted((b.offset, b.size, b.kind) for b in blocks)


@pytest.mark.parametrize("fv,ct,it,delta,meta", CASES)
def test_list_blocks_matches_writer(oracle, fv, ct, it, delta, meta):
    from speedb_amd import sst
    if fv == 0 and ct != 1:
        pytest.skip("format_version 0 implies kCRC32c")
    img, layout = write_sst(oracle, seed=fv * 31 + it, checksum_type=ct, format_version=fv, index_type=it,
                            delta=delta, meta=meta, n_data=37)
    f, blocks = sst.list_blocks(img)
    assert f.format_version == fv and f.checksum_type == ct
    assert f.index_type == it and bool(f.index_value_is_delta_encoded) == delta
    assert f.footer_offset == layout.footer_offset
    if fv >= 6:
        assert f.base_context_checksum == 0x5EED1234
    assert _kinds(blocks) == sorted(layout.blocks)
    # VerifyChecksum order: metaindex first, data blocks after the index
    assert blocks[0].kind == "metaindex"
    assert [b.offset for b in blocks if b.kind == "data"] == sorted(
        o for o, _, k in layout.blocks if k == "data")


def test_footer_errors(oracle):
    """Footer::DecodeFrom's corruption messages (table/format.cc:348-470)."""
    from speedb_amd import sst
    img, _ = write_sst(oracle, format_version=6, n_data=4)
    bad = bytearray(img)
    bad[-1] ^= 0xFF
    with pytest.raises(sst.SstError, match="Bad table magic number"):
        sst.list_blocks(bytes(bad))
    bad = bytearray(img)
    bad[-12:-8] = struct.pack("<I", 7)
    with pytest.raises(sst.SstError, match="Corrupt or unsupported format_version: 7"):
        sst.list_blocks(bytes(bad))
    bad = bytearray(img)
    bad[-53] = 9
    with pytest.raises(sst.SstError, match="Corrupt or unsupported checksum type: 9"):
        sst.list_blocks(bytes(bad))
    bad = bytearray(img)
    bad[-52] ^= 1
    with pytest.raises(sst.SstError, match="Bad extended magic number"):
        sst.list_blocks(bytes(bad))
    bad = bytearray(img)
    bad[-13] = 1  # checked reserved padding
    with pytest.raises(sst.SstError, match="future feature"):
        sst.list_blocks(bytes(bad))
    with pytest.raises(sst.SstError, match="too short"):
        sst.list_blocks(b"x" * 20)


def test_structure_errors(oracle):
    """A handle past the end of the file, a compressed index block."""
    from speedb_amd import sst
    img, layout = write_sst(oracle, format_version=5, n_data=6)
    f, blocks = sst.list_blocks(img)
    idx = next(b for b in blocks if b.kind == "index")
    bad = bytearray(img)
    bad[idx.offset + idx.size] = 1  # trailer type byte: compressed
    with pytest.raises(sst.SstError, match="compressed"):
        sst.list_blocks(bytes(bad))
    # truncate the file just before the footer: the metaindex handle dangles
    short = img[:idx.offset] + img[-53:]
    with pytest.raises(sst.SstError):
        sst.list_blocks(short)


@pytest.mark.gpu
@pytest.mark.parametrize("fv,ct,it,delta,meta", CASES)
def test_verify_sst_image(gpu, oracle, fv, ct, it, delta, meta):
    from speedb_amd import sst
    img, layout = write_sst(oracle, seed=fv * 7 + it, checksum_type=ct, format_version=fv, index_type=it,
                            delta=delta, meta=meta, n_data=53)
    per = []
    st = sst.VerifyChecksum(img, "000042.sst", per_block=per)
    assert st.ok(), st.ToString()
    assert len(per) == len(layout.blocks)
    if ct == 0:
        return  # kNoChecksum: nothing to corrupt
    # flip one byte in three blocks of different kinds: exactly those fail
    f, blocks = sst.list_blocks(img)
    rnd = random.Random(fv)
    victims = [rnd.choice([b for b in blocks if b.kind == "data"]),
               next(b for b in blocks if b.kind == "properties")]
    bad = bytearray(img)
    for b in victims:
        bad[b.offset + b.size // 2] ^= 0x10
    per = []
    st = sst.VerifyChecksum(bytes(bad), "000042.sst", per_block=per)
    assert st.IsCorruption()
    assert "block checksum mismatch" in st.message and "in 000042.sst offset" in st.message
    failed = sorted(b.offset for b, s in per if not s.ok())
    assert failed == sorted(b.offset for b in victims)


@pytest.mark.gpu
def test_verify_sst_footer_checksum(gpu, oracle):
    """format_version 6: a flipped bit in the footer's reserved (unchecked)
    padding is caught by the footer checksum (table/format.cc:419-426)."""
    from speedb_amd import sst
    img, _ = write_sst(oracle, format_version=6, n_data=5, checksum_type=4)
    assert sst.VerifyChecksum(img).ok()
    bad = bytearray(img)
    bad[-53 + 1 + 16 + 3] ^= 0x40  # inside the 16 unchecked reserved bytes
    st = sst.VerifyChecksum(bytes(bad))
    assert st.IsCorruption() and "checksum mismatch" in st.message and "Footer at" in st.message


@pytest.mark.parametrize("index_type", [0, 2])
def test_compressed_index_is_not_parsed(oracle, index_type):
    """An index block with a compression type (enable_index_compression, on
    by default -- include/rocksdb/table.h:541) cannot be read by the host
    lister (no decompressor): NotSupported, never a wrong block list."""
    from speedb_amd import sst
    img, _ = write_sst(oracle, format_version=5, index_type=index_type, n_data=20, index_comp=1)
    with pytest.raises(sst.SstError) as e:
        sst.list_blocks(img)
    assert e.value.rc == sst.MCK_ENOTSUP and e.value.status.code == "Not implemented"
    assert "compressed" in str(e.value)


@pytest.mark.parametrize("fv,it,delta", [(2, 0, False), (5, 0, True), (5, 2, True), (6, 2, True), (6, 3, False),
                                         (4, 1, True)])
def test_compressed_index_listed_through_callback(oracle, fv, it, delta):
    """Tables with zlib-compressed index blocks (and, two-level, compressed
    partitions): mck_sst_list_blocks_uncompress hands every compressed block
    the lister reads to the caller's callback -- here the inverse of the
    reference's Zlib_Compress format; in an integration its
    UncompressBlockData -- and lists exactly the blocks the writer wrote,
    with their STORED (compressed) handles."""
    from sst_format import zlib_unblock
    from speedb_amd import sst
    img, layout = write_sst(oracle, seed=fv * 13 + it, format_version=fv, index_type=it, delta=delta, n_data=33,
                            index_comp=2, meta=("filter", "range_del"))
    with pytest.raises(sst.SstError) as e:  # no callback: as before
        sst.list_blocks(img)
    assert e.value.rc == sst.MCK_ENOTSUP
    seen = []

    def unz(t, off, raw):
        assert t == 2
        seen.append(off)
        return zlib_unblock(raw)

    f, blocks = sst.list_blocks(img, uncompress=unz)
    assert _kinds(blocks) == sorted(layout.blocks)
    assert f.index_type == it and bool(f.index_value_is_delta_encoded) == delta
    idx = sorted(o for o, _, k in layout.blocks if k in ("index", "index_partition"))
    # every compressed index block, once per pass (list_blocks: count, then list)
    assert sorted(set(seen)) == idx and len(seen) == 2 * len(idx)


def test_compressed_index_callback_errors(oracle):
    """A failing callback (an exception in Python; any non-OK return in C)
    fails the listing with the callback's code, naming the block."""
    from speedb_amd import sst
    img, layout = write_sst(oracle, format_version=5, index_type=2, n_data=20, index_comp=2)

    def bad(t, off, raw):
        raise ValueError("codec missing")

    with pytest.raises(sst.SstError) as e:
        sst.list_blocks(img, uncompress=bad)
    assert e.value.rc == sst.MCK_ECORRUPT and "uncompress callback failed" in str(e.value)
    # garbage "uncompressed" contents are parsed and rejected as a bad index
    with pytest.raises(sst.SstError) as e:
        sst.list_blocks(img, uncompress=lambda t, off, raw: b"\xff" * 7)
    assert e.value.rc == sst.MCK_ECORRUPT


@pytest.mark.parametrize("delta,it", [(False, 0), (True, 0), (True, 3), (False, 3)])
def test_index_handles_of_one_block(delta, it):
    """mck_sst_index_handles: the handles an already-uncompressed index block
    lists (IndexBlockIter), full or delta-encoded values, with first keys."""
    from sst_format import index_block
    from speedb_amd import sst
    rnd = random.Random(7)
    hs, off = [], 0
    for _ in range(70):
        n = rnd.randrange(100, 9000)
        hs.append((off, n))
        off += n + 5
    keys = [b"k%06d" % (3 * i + 1) for i in range(len(hs))]
    fks = [b"k%06d" % (3 * i) for i in range(len(hs))] if it == 3 else None
    blk = index_block(hs, keys, delta, 4, fks)
    got = sst.index_handles(blk, delta, it, "data")
    assert [(b.offset, b.size, b.kind) for b in got] == [(o, n, "data") for o, n in hs]
    top = sst.index_handles(blk, delta, it, "index_partition")
    assert all(b.kind == "index_partition" for b in top)
    with pytest.raises(sst.SstError):
        sst.index_handles(blk[:-9], delta, it)


@pytest.mark.gpu
@pytest.mark.parametrize("fv,index_type", [(5, 2), (6, 0)])
def test_compressed_index_whole_file_verify(gpu, oracle, fv, index_type):
    """VerifyChecksum of a table with zlib-compressed index blocks: listed
    through the callback, every block (the compressed ones included)
    verified in one GPU batch; a flipped byte in a compressed partition is
    flagged at exactly that block."""
    from sst_format import zlib_unblock
    from speedb_amd import sst
    img, layout = write_sst(oracle, format_version=fv, index_type=index_type, n_data=40, index_comp=2)
    unz = lambda t, off, raw: zlib_unblock(raw)  # noqa: E731
    per = []
    st = sst.VerifyChecksum(img, "000011.sst", per_block=per, uncompress=unz)
    assert st.ok(), st.ToString()
    assert sorted((b.offset, b.size, b.kind) for b, _ in per) == sorted(layout.blocks)
    tgt = [h for h in sorted(layout.blocks) if h[2] == ("index_partition" if index_type == 2 else "index")][-1]
    bad = bytearray(img)
    bad[tgt[0] + tgt[1]] ^= 0x40  # the stored trailer's type byte: the checksum covers it
    per = []
    st = sst.VerifyChecksum(bytes(bad), "000011.sst", per_block=per,
                            uncompress=lambda t, off, raw: zlib_unblock(raw) if t == 2 else
                            (_ for _ in ()).throw(ValueError(t)))
    assert not st.ok()


@pytest.mark.gpu
@pytest.mark.parametrize("fv,index_type", [(5, 0), (6, 2)])
def test_compressed_index_low_level_verify(gpu, oracle, fv, index_type):
    """The documented path for such tables: the reader's
    own IndexBlockIter / metaindex walk names the blocks, one GPU batch
    verifies all of them -- the compressed index blocks included (the
    checksum covers the stored bytes and the type byte)."""
    import speedb_amd as S
    from speedb_amd import sst
    img, layout = write_sst(oracle, format_version=fv, index_type=index_type, n_data=30, index_comp=1,
                            meta=("filter", "range_del"))
    handles = sorted(layout.blocks)
    per = []
    st = sst.VerifyBlocks(img, handles, 1, 0x5EED1234 if fv >= 6 else 0, "000007.sst", per_block=per)
    assert st.ok(), st.ToString()
    assert len(per) == len(handles) and all(s.ok() for _, s in per)
    assert any(k == "index" for _, _, k in handles)
    # a flipped byte in the compressed index block and in one data block
    bad = bytearray(img)
    idx = [h for h in handles if h[2] == "index"][0]
    dat = [h for h in handles if h[2] == "data"][7]
    bad[idx[0] + 3] ^= 0x10
    bad[dat[0] + dat[1]] ^= 0x01  # the type byte
    per = []
    st = sst.VerifyBlocks(bytes(bad), handles, 1, 0x5EED1234 if fv >= 6 else 0, "000007.sst", per_block=per)
    assert st.IsCorruption() and "block checksum mismatch" in st.ToString()
    assert sorted(b.offset for b, s in per if not s.ok()) == sorted([idx[0], dat[0]])

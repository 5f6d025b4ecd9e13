"""Blob files: the host walk lists exactly the records
the test-side writer produced and reports the reference's header errors;
on the GPU every record's header and blob CRC verifies in one batch,
injected corruption is flagged per record with the reference's messages,
and the write side reproduces the writer's CRC fields bit-exactly."""
import struct

import pytest

from blob_format import blob_file


def test_list_records(oracle):
    from speedb_amd import blob
    img, recs = blob_file(oracle, n_records=40, seed=3)
    info, got = blob.list_records(img)
    assert info.version == 1 and info.column_family_id == 7 and info.has_footer
    assert info.footer_blob_count == 40
    assert [(r.offset, r.key_size, r.value_size) for r in got] == recs
    img2, recs2 = blob_file(oracle, n_records=5, seed=4, footer=False)
    info2, got2 = blob.list_records(img2)
    assert not info2.has_footer and len(got2) == 5


def test_header_errors(oracle):
    from speedb_amd import blob
    img, _ = blob_file(oracle, n_records=3)
    bad = bytearray(img)
    bad[0] ^= 1
    with pytest.raises(blob.BlobError, match="Error while decoding blob log header: Magic number mismatch"):
        blob.list_records(bytes(bad))
    bad = bytearray(img)
    bad[4] = 2
    with pytest.raises(blob.BlobError, match="Unknown header version"):
        blob.list_records(bytes(bad))
    with pytest.raises(blob.BlobError, match="Unexpected blob file header size"):
        blob.list_records(img[:20])
    # a record whose value size runs past the end
    bad = bytearray(img)
    struct.pack_into("<Q", bad, 30 + 8, 1 << 40)
    with pytest.raises(blob.BlobError, match="past the end"):
        blob.list_records(bytes(bad))


@pytest.mark.gpu
def test_verify_blob_file(gpu, oracle):
    from speedb_amd import blob
    img, recs = blob_file(oracle, n_records=300, seed=5, sizes=(0, 20000))
    per = []
    assert blob.VerifyBlobFile(img, per_record=per).ok()
    assert len(per) == 300
    bad = bytearray(img)
    bad[recs[10][0] + 16] ^= 1                      # expiration: header CRC
    bad[recs[20][0] + 32 + 2] ^= 1                  # key byte: blob CRC
    o, k, v = recs[30]
    bad[o + 32 + k + v // 2 if v else o + 32] ^= 1  # value byte: blob CRC
    per = []
    st = blob.VerifyBlobFile(bytes(bad), per_record=per)
    assert st.IsCorruption() and "Header CRC mismatch" in st.message
    msgs = {r.offset: s.message for r, s in per if not s.ok()}
    assert set(msgs) == {recs[10][0], recs[20][0], recs[30][0]}
    assert "Header CRC mismatch" in msgs[recs[10][0]]
    assert msgs[recs[20][0]] == "Blob CRC mismatch" == msgs[recs[30][0]]
    bad = bytearray(img)
    bad[-5] ^= 1  # footer expiration range: footer CRC
    assert "footer: CRC mismatch" in blob.VerifyBlobFile(bytes(bad)).message


@pytest.mark.gpu
def test_write_record_crcs(gpu, oracle):
    """BlobLogRecord::EncodeHeaderTo on the device: zeroed CRC fields are
    recomputed bit-exactly."""
    import torch

    from speedb_amd import blob
    img, recs = blob_file(oracle, n_records=200, seed=6, sizes=(0, 5000))
    blank = bytearray(img)
    for o, _, _ in recs:
        blank[o + 24:o + 32] = bytes(8)
    info, got = blob.list_records(bytes(blank))
    dev, offs, lens = blob._device_records(bytes(blank), got, torch.device("cuda"))
    blob.WriteRecordCrcs(dev, offs, lens)
    assert bytes(dev[:len(img)].cpu().numpy().tobytes()) == img


@pytest.mark.gpu
def test_record_batch_large_static_feed(gpu, oracle):
    """More records than a workgroup's LDS descriptor cache (> 393,216 on 256
    CUs: the static feed, whose first span per wave has a wave-uniform
    address) with headers at odd byte offsets and one-round blobs: the
    header fields must be read with vector loads (a scalar 16-byte load drops
    the low address bits).  Write side vs the oracle, then verify."""
    import numpy as np
    import torch
    from speedb_amd import blob
    n, kb, vb = 420_000, 16, 200
    rec = 32 + kb + vb
    g = torch.Generator(device="cuda")
    g.manual_seed(11)
    img = torch.randint(0, 256, (30 + n * rec + 64,), dtype=torch.uint8, device="cuda", generator=g)
    recs = img[30:30 + n * rec].view(n, rec)
    recs[:, 0:8] = torch.tensor(list(kb.to_bytes(8, "little")), dtype=torch.uint8, device="cuda")
    recs[:, 8:16] = torch.tensor(list(vb.to_bytes(8, "little")), dtype=torch.uint8, device="cuda")
    offs = 30 + torch.arange(n, dtype=torch.int64, device="cuda") * rec
    lens = torch.full((n,), kb + vb, dtype=torch.int32, device="cuda")
    blob.WriteRecordCrcs(img, offs, lens)
    h = img.cpu().numpy().tobytes()
    for i in list(range(0, 8192)) + list(range(8192, n, 101)) + [n - 1]:
        o = 30 + i * rec
        assert struct.unpack_from("<I", h, o + 24)[0] == oracle.Mask(oracle.Value(h[o:o + 24])), i
        assert struct.unpack_from("<I", h, o + 28)[0] == oracle.Mask(oracle.Value(h[o + 32:o + rec])), i
    st = blob.record_batch(False, img, offs, lens)
    assert int(st.sum().item()) == 0
    img[30 + 5 * rec + 40] ^= 1  # one blob byte of record 5
    st = blob.record_batch(False, img, offs, lens).cpu().numpy()
    assert np.nonzero(st)[0].tolist() == [5] and st[5] == 2

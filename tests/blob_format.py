"""Test-side blob file writer -- TEST INFRASTRUCTURE.  Restates
BlobLogWriter's layout (db/blob/blob_log_writer.cc, blob_log_format.cc:14-25
header, :57-68 footer, :97-112 record header) with CRCs from the CPU oracle."""
import random
import struct

MAGIC = 2395959


def blob_file(oracle, n_records=50, seed=1, footer=True, sizes=(0, 9000), cf=7, ttl=False):
    rnd = random.Random(seed)
    out = bytearray(struct.pack("<IIIBBQQ", MAGIC, 1, cf, 1 if ttl else 0, 0, 10, 20))
    recs = []
    for i in range(n_records):
        key = b"blobkey%06d" % i
        value = bytes(rnd.getrandbits(8) for _ in range(rnd.randrange(*sizes)))
        hdr = struct.pack("<QQQ", len(key), len(value), 1000 + i)
        hcrc = oracle.Mask(oracle.Value(hdr))
        bcrc = oracle.Mask(oracle.Extend(oracle.Value(key), value))
        recs.append((len(out), len(key), len(value)))
        out += hdr + struct.pack("<II", hcrc, bcrc) + key + value
    if footer:
        f = struct.pack("<IQQQ", MAGIC, n_records, 10, 20)
        out += f + struct.pack("<I", oracle.Mask(oracle.Value(f)))
    return bytes(out), recs

"""Pin the CPU oracle (oracle/oracle.c) against the reference: its own
known-answer tests (tests/golden/kat.json), the fixtures generated from the
compiled reference (tests/golden/vectors.json), and -- when oracle/_ref was
built -- a live differential run against the reference library."""
import os
import random
import struct

import pytest

from formats import WalWriter, folly_buffer, wal_expected_blocks


def _hx(v):
    return struct.pack("<I", v).hex().upper()


def test_rfc3720_vectors(oracle, golden):
    kat = {r["pattern"]: int(r["crc"], 16) for r in golden["kat"]["rfc3720"]}
    assert oracle.Value(bytes(32)) == kat["zeros32"]
    assert oracle.Value(b"\xff" * 32) == kat["ff32"]
    assert oracle.Value(bytes(range(32))) == kat["inc32"]
    assert oracle.Value(bytes(31 - i for i in range(32))) == kat["dec32"]
    assert oracle.Value(bytes.fromhex(golden["kat"]["iscsi48"])) == kat["iscsi48"]


@pytest.mark.slow
def test_folly_3way_vectors(oracle, golden):
    buf = folly_buffer(golden["kat"]["folly_buffer_bytes"])
    for off, n, expected in golden["kat"]["folly"]:
        # util/crc32c_test.cc:96-111 compares against ~expected
        assert oracle.Value(buf[off:off + n]) == (~expected) & 0xFFFFFFFF
        half = n // 2
        part = oracle.Value(buf[off:off + half])
        assert oracle.Extend(part, buf[off + half:off + n]) == (~expected) & 0xFFFFFFFF


def test_crc_api_semantics(oracle):
    # util/crc32c_test.cc:113-171
    assert oracle.Value(b"a") != oracle.Value(b"foo")
    assert oracle.Value(b"hello world") == oracle.Extend(oracle.Value(b"hello "), b"world")
    c = oracle.Value(b"foo")
    assert c != oracle.Mask(c) and c != oracle.Mask(oracle.Mask(c))
    assert oracle.Unmask(oracle.Mask(c)) == c
    assert oracle.Unmask(oracle.Unmask(oracle.Mask(oracle.Mask(c)))) == c
    c1, c2, c3 = oracle.Value(b"hello "), oracle.Value(b"world"), oracle.Value(b"hello world")
    assert oracle.Combine(c1, c2, 5) == c3
    assert oracle.Combine(c2, c1, 6) != c3
    rnd = random.Random(7)
    s1 = bytes(rnd.getrandbits(8) for _ in range(1 << 16))
    crc1 = oracle.Value(s1)
    for n in list(range(0, 300)) + [4096, 65537]:
        s2 = bytes(rnd.getrandbits(8) for _ in range(n))
        assert oracle.Combine(crc1, oracle.Value(s2), n) == oracle.Extend(crc1, s2)


def test_checksum_schemas(oracle, golden):
    """table/table_test.cc:2286-2403 BuiltinChecksumTest.ChecksumSchemas."""
    si = golden["kat"]["schemas_inputs"]
    b0 = si["b0"].encode()
    b1 = si["b1"].encode()
    b2 = (si["b2_repeat"] * si["b2_times"] + si["b2_suffix"]).encode()
    cts = [si["compression_last_bytes"][k] for k in ("ct1", "ct2", "ct3")]
    for t, exp in golden["kat"]["schemas"].items():
        t = int(t)
        assert _hx(oracle.Builtin(t, b"")) == exp["empty"]
        for name, data in (("b0", b0), ("b1", b1), ("b2", b2)):
            for ct, want in zip(cts, exp[name]):
                d = data[:-1] + bytes([ct])
                v = oracle.Builtin(t, d)
                assert _hx(v) == want, (t, name, ct)
                # table_test.cc:2297-2300: consistency with WithLastByte
                assert oracle.BuiltinLast(t, d[:-1], d[-1]) == v


def test_checksum_zero_inputs(oracle):
    """table/table_test.cc:2405-2440 (strided subset of lengths < 20000)."""
    zeros = bytes(20000)
    lens = list(range(0, 1100)) + list(range(1100, 20000, 97))
    for t in (1, 2, 3, 4):
        for n in lens:
            v = oracle.Builtin(t, zeros[:n])
            if v == 0:
                assert t == 4 and n == 0, (t, n)


def test_survey_extra_values(oracle, golden):
    e = golden["kat"]["survey_extra"]
    for n, key in ((4096, "x4096"), (16384, "x16384"), (65536, "x65536")):
        d = b"x" * n
        assert oracle.Value(d) == int(e[key]["crc"], 16)
        assert oracle.Mask(oracle.Value(d)) == int(e[key]["masked"], 16)
        assert oracle.XXH3(d) == int(e[key]["xxh3"], 16)
    assert oracle.Value(b"123456789") == int(e["123456789"]["crc"], 16)
    assert oracle.XXH3(b"123456789") == int(e["123456789"]["xxh3"], 16)
    cm = e["context_modifier"]
    assert oracle.ContextModifier(int(cm["base"], 16), int(cm["offset"], 16)) == int(cm["out"], 16)
    for t, want in zip(range(1, 6), e["wal_type_crc_1_to_5"]):
        assert oracle.Value(bytes([t])) == int(want, 16)


def test_vectors_from_reference(oracle, golden):
    blob = golden["blob"]
    for c in golden["cases"]:
        d = blob[c["off"]:c["off"] + c["len"]]
        assert oracle.Value(d) == c["crc32c"], c["len"]
        assert oracle.Extend(c["extend_init"], d) == c["crc32c_extend"]
        assert oracle.XXH3(d) == c["xxh3"], c["len"]
        assert oracle.XXH32(d) == c["xxh32"]
        assert oracle.XXH64(d) == c["xxh64"]
        for t, v in c["builtin"].items():
            assert oracle.Builtin(int(t), d) == v, (t, c["len"])
            if d:
                assert oracle.BuiltinLast(int(t), d[:-1], d[-1]) == v
    for c in golden["combine"]:
        assert oracle.Combine(c["crc1"], c["crc2"], c["len2"]) == c["out"]
    for c in golden["context_modifier"]:
        assert oracle.ContextModifier(c["base"], c["offset"]) == c["out"]
    for c in golden["wal_records"]:
        d = blob[c["off"]:c["off"] + c["len"]]
        assert oracle.WalRecordCrc(c["type"], d, c["recyclable"], c["log_number"]) == c["crc"]
    for t, v in enumerate(golden["wal_type_crc"]):
        assert oracle.Value(bytes([t])) == v


def test_hash64_small_value_schema(oracle, golden):
    """util/hash_test.cc:162-228: Hash64 (XXPH3, seed 0) of short strings."""
    for h, v in golden["kat"]["hash64_small"]:
        assert oracle.Hash64(bytes.fromhex(h)) == int(v), h


def test_hash64_large_value_schema(oracle, golden):
    """util/hash_test.cc:216-279: the mod-61 descriptor of Hash64 over every
    prefix length < 430 of a repeated string (covers all XXPH3 length classes
    up to the long loop)."""
    enc = "abcdefghijklmnopqrstuvwxyz123456789ABCDEFGHIJKLMNOPQRSTUVWXYZ"
    for rep, want in golden["kat"]["hash64_descriptors"].items():
        inp = (rep * 430)[:430].encode()
        got = "".join(enc[oracle.Hash64(inp[:i]) % 61] for i in range(430))
        assert got == want, rep


def test_hash64_and_kv_protect_vectors(oracle, golden):
    blob = golden["blob"]
    for c in golden["hash64"]:
        d = blob[c["off"]:c["off"] + c["len"]]
        assert oracle.Hash64(d, c["seed"]) == c["out"], (c["len"], c["seed"])
    for c in golden["kv_protect"]:
        k = blob[c["koff"]:c["koff"] + c["klen"]]
        v = blob[c["voff"]:c["voff"] + c["vlen"]]
        assert oracle.KvProtect(c["mode"], k, v, c["op"], c["extra"]) == c["out"]


def test_oracle_vs_live_reference(oracle, ref):
    if ref is None:
        pytest.skip("oracle/_ref not built")
    rnd = random.Random(99)
    for _ in range(300):
        n = rnd.choice([rnd.randrange(0, 300), rnd.randrange(0, 70000)])
        d = os.urandom(n)
        init = rnd.getrandbits(32)
        assert oracle.Extend(init, d) == ref.ref_crc32c_extend(init, d, n)
        assert oracle.XXH3(d) == ref.ref_xxh3_64(d, n)
        assert oracle.XXH32(d, 5) == ref.ref_xxh32(d, n, 5)
        assert oracle.XXH64(d, 9) == ref.ref_xxh64(d, n, 9)
        for t in range(5):
            assert oracle.Builtin(t, d) == ref.ref_builtin_checksum(t, d, n)
        seed = rnd.choice([0, rnd.getrandbits(64)])
        assert oracle.Hash64(d, seed) == ref.ref_hash64(d, n, seed)
    # table/format.h ChecksumModifierForContext, called from the reference header
    for _ in range(20000):
        base = rnd.choice([0, 1, rnd.getrandbits(32)])
        off = rnd.getrandbits(rnd.choice([8, 32, 33, 64]))
        assert oracle.ContextModifier(base, off) == ref.ref_context_modifier(base, off)


def test_wal_writer_layout(oracle):
    """Restated AddRecord: fragments never straddle a 32 KiB block, the block
    tail < header is zero padded, and every record verifies."""
    for recycle in (False, True):
        w = WalWriter(oracle, log_number=123, recycle=recycle)
        rnd = random.Random(3)
        for n in [0, 1, 100, 32761, 32762, 70000, 5, 32750, 12]:
            w.add_record(bytes(rnd.getrandbits(8) for _ in range(n)))
        data = bytes(w.buf)
        for off, t, n in w.records:
            hs = 11 if recycle else 7
            assert off // 32768 == (off + hs + n - 1) // 32768 or n == 0
        exp = wal_expected_blocks(data, 123, oracle)
        assert all(s == 0 for _, s, _, _ in exp), exp
        assert sum(r for r, _, _, _ in exp) == len(w.records)


def test_oracle_file_checksum_crc32c(oracle, ref):
    """FileChecksumGenCrc32c restatement: big-endian Value of the whole file
    (util/file_checksum_helper.h:22-46), pinned to the crc32c_test.cc:81
    vector and to the reference's crc32c::Value on random files."""
    import random
    assert oracle.FileChecksumCrc32c(b"123456789") == bytes.fromhex("e3069283")
    assert oracle.FileChecksumCrc32c(b"") == bytes(4)
    rnd = random.Random(5)
    for n in (1, 4096, 65537, 300001):
        b = bytes(rnd.getrandbits(8) for _ in range(n))
        want = ref.ref_crc32c_value(b, n) if ref is not None else oracle.Value(b)
        assert oracle.FileChecksumCrc32c(b) == want.to_bytes(4, "big")

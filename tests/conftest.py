"""Shared fixtures.

* ``oracle``  -- ctypes handle on oracle/liboracle.so, the CPU restatement of
  the reference checksum path (TEST INFRASTRUCTURE; built on demand with make).
* ``ref``     -- ctypes handle on oracle/_ref/libspdb_ref.so (the reference's
  own util/crc32c.cc + util/xxhash.cc + util/hash.cc), or None when it was
  not built.
* ``golden``  -- tests/golden/vectors.json + blob.bin + kat.json.

Tests that need a GPU carry ``@pytest.mark.gpu``.
"""
import ctypes
import json
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
GOLDEN = os.path.join(REPO, "tests", "golden")


# Child pytest processes of the forced-driver tests set these; the engine
# itself reads no environment (mck_test_set_crc_driver / mck_test_set_xxh3_driver
# are its test hooks).
CRC_DRIVERS = {"rows16": 2, "rows8": 3, "rows4": 5, "rows1": 6, "bh": 7, "small": 9}


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running")
    drv = os.environ.get("SPEEDB_AMD_TEST_CRC_DRIVER")
    order = os.environ.get("SPEEDB_AMD_TEST_CRC_ORDER")
    x3 = os.environ.get("SPEEDB_AMD_TEST_X3_DRIVER")
    if drv or order or x3:
        import sys
        if REPO not in sys.path:
            sys.path.insert(0, REPO)
        # torch's HIP runtime first, as in every other process (the gpu
        # fixture initialises torch before it imports speedb_amd): a child
        # that loaded the engine first saw mck_device_count() == 0
        import torch
        torch.cuda.is_available()
        from speedb_amd import _lib
        _lib.check(_lib.lib.mck_test_set_crc_driver(CRC_DRIVERS.get(drv, 0), 1 if order == "interleaved" else 0),
                   "mck_test_set_crc_driver")
        _lib.check(_lib.lib.mck_test_set_xxh3_driver({"wave": 1, "rows": 2}.get(x3, 0)), "mck_test_set_xxh3_driver")


def _bind(lib, prefix):
    c = ctypes
    sig = {
        "crc32c_extend": (c.c_uint32, [c.c_uint32, c.c_char_p, c.c_size_t]),
        "crc32c_value": (c.c_uint32, [c.c_char_p, c.c_size_t]),
        "crc32c_mask": (c.c_uint32, [c.c_uint32]),
        "crc32c_unmask": (c.c_uint32, [c.c_uint32]),
        "crc32c_combine": (c.c_uint32, [c.c_uint32, c.c_uint32, c.c_size_t]),
        "xxh3_64": (c.c_uint64, [c.c_char_p, c.c_size_t]),
        "xxh32": (c.c_uint32, [c.c_char_p, c.c_size_t, c.c_uint32]),
        "xxh64": (c.c_uint64, [c.c_char_p, c.c_size_t, c.c_uint64]),
        "builtin_checksum": (c.c_uint32, [c.c_int, c.c_char_p, c.c_size_t]),
        "wal_record_crc": (c.c_uint32, [c.c_uint8, c.c_char_p, c.c_size_t, c.c_int, c.c_uint32]),
    }
    if prefix == "orc":
        sig.update({
            "crc32c_zshift": (c.c_uint32, [c.c_uint32, c.c_uint64]),
            "builtin_checksum_with_last_byte": (c.c_uint32, [c.c_int, c.c_char_p, c.c_size_t,
                                                             c.c_uint8]),
            "file_checksum_crc32c": (None, [c.c_char_p, c.c_size_t, c.c_char_p]),
            "verify_block": (c.c_int, [c.c_int, c.c_char_p, c.c_size_t, c.c_uint32, c.c_uint64,
                                       ctypes.POINTER(c.c_uint32), ctypes.POINTER(c.c_uint32)]),
            "block_kv_protect": (c.c_int, [c.c_int, c.c_char_p, c.c_size_t, c.c_uint32, c.c_char_p,
                                           c.c_size_t, ctypes.POINTER(c.c_uint32),
                                           ctypes.POINTER(c.c_uint32)]),
        })
    sig.update({
        "context_modifier": (c.c_uint32, [c.c_uint32, c.c_uint64]),
        "hash64": (c.c_uint64, [c.c_char_p, c.c_size_t, c.c_uint64]),
        "kv_protect": (c.c_uint64, [c.c_int, c.c_char_p, c.c_size_t, c.c_char_p, c.c_size_t,
                                    c.c_uint8, c.c_uint64]),
    })
    for name, (res, args) in sig.items():
        f = getattr(lib, f"{prefix}_{name}")
        f.restype, f.argtypes = res, args
    return lib


class _Oracle:
    """Pythonic wrapper; names follow the reference."""

    def __init__(self, lib):
        self.lib = lib

    def Value(self, b):
        return self.lib.orc_crc32c_value(b, len(b))

    def Extend(self, init, b):
        return self.lib.orc_crc32c_extend(init, b, len(b))

    def Mask(self, v):
        return self.lib.orc_crc32c_mask(v)

    def Unmask(self, v):
        return self.lib.orc_crc32c_unmask(v)

    def Combine(self, a, b, n):
        return self.lib.orc_crc32c_combine(a, b, n)

    def XXH3(self, b):
        return self.lib.orc_xxh3_64(b, len(b))

    def XXH32(self, b, seed=0):
        return self.lib.orc_xxh32(b, len(b), seed)

    def XXH64(self, b, seed=0):
        return self.lib.orc_xxh64(b, len(b), seed)

    def Builtin(self, t, b):
        return self.lib.orc_builtin_checksum(int(t), b, len(b))

    def BuiltinLast(self, t, b, last):
        return self.lib.orc_builtin_checksum_with_last_byte(int(t), b, len(b), last)

    def ContextModifier(self, base, off):
        return self.lib.orc_context_modifier(base, off)

    def FileChecksumCrc32c(self, b):
        out = ctypes.create_string_buffer(4)
        self.lib.orc_file_checksum_crc32c(b, len(b), out)
        return out.raw

    def Hash64(self, b, seed=0):
        return self.lib.orc_hash64(b, len(b), seed)

    def KvProtect(self, mode, key, value, op=0, extra=0):
        return self.lib.orc_kv_protect(mode, key, len(key), value, len(value), op, extra)

    def BlockKvProtect(self, kind, block, prot_bytes):
        """(status, kv_checksum bytes, restart interval) of one block
        (block.cc:1091-1222 Initialize*BlockProtectionInfo)."""
        nk, ri = ctypes.c_uint32(), ctypes.c_uint32()
        cap = len(block) * 8 + 64
        out = ctypes.create_string_buffer(cap)
        st = self.lib.orc_block_kv_protect(int(kind), block, len(block), prot_bytes, out, cap,
                                           ctypes.byref(nk), ctypes.byref(ri))
        assert nk.value * prot_bytes <= cap
        return st, out.raw[:nk.value * prot_bytes], ri.value

    def WalRecordCrc(self, t, payload, recyclable, log_number):
        return self.lib.orc_wal_record_crc(t, payload, len(payload), 1 if recyclable else 0,
                                           log_number & 0xFFFFFFFF)


@pytest.fixture(scope="session")
def oracle():
    so = os.path.join(ORACLE_DIR, "liboracle.so")
    src = os.path.join(ORACLE_DIR, "oracle.c")
    if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", ORACLE_DIR, so])
    return _Oracle(_bind(ctypes.CDLL(so), "orc"))


@pytest.fixture(scope="session")
def ref():
    so = os.path.join(ORACLE_DIR, "_ref", "libspdb_ref.so")
    if not os.path.exists(so):
        return None
    return _bind(ctypes.CDLL(so), "ref")


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(GOLDEN, "vectors.json")) as f:
        v = json.load(f)
    with open(os.path.join(GOLDEN, "blob.bin"), "rb") as f:
        v["blob"] = f.read()
    with open(os.path.join(GOLDEN, "kat.json")) as f:
        v["kat"] = json.load(f)
    return v


@pytest.fixture(scope="session")
def gpu():
    """torch + speedb_amd on cuda:0; skips when no GPU is visible."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import speedb_amd
    assert speedb_amd.device_count() >= 1, "GPU visible to torch but not a gfx950 device"
    return torch

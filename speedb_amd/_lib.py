"""ctypes binding of the engine's C ABI (include/speedb_amd/mck.h).

The shared library ``speedb_amd/libspeedb_amd.so`` is built in-tree by
``__graft_entry__.build()`` (hipcc, gfx950).  There is no CPU fallback: if the
library is missing, importing this module raises.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
DEFAULT_LIB_PATH = os.path.join(_HERE, "libspeedb_amd.so")
# An alternative build of the same engine (A/B experiments under microbench/,
# `bench.py --engine-lib PATH`) is loaded only when BOTH SPEEDB_AMD_LIB names
# it and SPEEDB_AMD_AB=1 says so: a stray SPEEDB_AMD_LIB in a production
# environment is refused instead of silently swapping the engine.
_OVERRIDE = os.environ.get("SPEEDB_AMD_LIB")
AB_MODE = os.environ.get("SPEEDB_AMD_AB") == "1"
if _OVERRIDE and not AB_MODE:
    raise ImportError(
        f"speedb_amd: SPEEDB_AMD_LIB={_OVERRIDE} is set without SPEEDB_AMD_AB=1; an alternative engine "
        "build is loaded only for explicit A/B runs (bench.py --engine-lib PATH)")
LIB_PATH = _OVERRIDE if _OVERRIDE else DEFAULT_LIB_PATH

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"speedb_amd: native engine {LIB_PATH} is missing; run "
        "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950). "
        "There is no CPU fallback.")

lib = ctypes.CDLL(LIB_PATH)


def lib_identity() -> dict:
    """Path and sha256 of the engine this process loaded (recorded in every
    bench line, so a number names the exact .so it timed)."""
    h = hashlib.sha256()
    with open(LIB_PATH, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return {"path": os.path.relpath(LIB_PATH, os.path.dirname(_HERE)) if LIB_PATH.startswith(os.path.dirname(_HERE))
            else LIB_PATH, "sha256": h.hexdigest(), "override": bool(_OVERRIDE)}

u8p = ctypes.POINTER(ctypes.c_uint8)
u32p = ctypes.POINTER(ctypes.c_uint32)
u64p = ctypes.POINTER(ctypes.c_uint64)
vp = ctypes.c_void_p


class mck_spans(ctypes.Structure):
    _fields_ = [
        ("base", vp),
        ("offsets", vp),
        ("lengths", vp),
        ("stride", ctypes.c_uint64),
        ("length", ctypes.c_uint32),
        ("count", ctypes.c_uint32),
    ]


class mck_wal_block_result(ctypes.Structure):
    _fields_ = [
        ("records_ok", ctypes.c_uint32),
        ("status", ctypes.c_int32),
        ("stop_offset", ctypes.c_uint32),
        ("bytes_ok", ctypes.c_uint32),
    ]


# (name, restype, argtypes) for every symbol declared in mck.h
SIGNATURES = [
    ("mck_last_error", ctypes.c_char_p, []),
    ("mck_version", ctypes.c_char_p, []),
    ("mck_device_count", ctypes.c_int, []),
    ("mck_crc32c_mask", ctypes.c_uint32, [ctypes.c_uint32]),
    ("mck_crc32c_unmask", ctypes.c_uint32, [ctypes.c_uint32]),
    ("mck_crc32c_combine", ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_size_t]),
    ("mck_context_modifier", ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_uint64]),
    ("mck_crc32c_extend", ctypes.c_uint32, [ctypes.c_uint32, vp, ctypes.c_size_t]),
    ("mck_crc32c_value", ctypes.c_uint32, [vp, ctypes.c_size_t]),
    ("mck_xxh3_64", ctypes.c_uint64, [vp, ctypes.c_size_t]),
    ("mck_builtin_checksum", ctypes.c_uint32, [ctypes.c_int, vp, ctypes.c_size_t]),
    ("mck_builtin_checksum_with_last_byte", ctypes.c_uint32,
     [ctypes.c_int, vp, ctypes.c_size_t, ctypes.c_char]),
    ("mck_crc32c_extend_r", ctypes.c_int, [ctypes.c_uint32, vp, ctypes.c_size_t, u32p]),
    ("mck_crc32c_value_r", ctypes.c_int, [vp, ctypes.c_size_t, u32p]),
    ("mck_xxh3_64_r", ctypes.c_int, [vp, ctypes.c_size_t, u64p]),
    ("mck_builtin_checksum_r", ctypes.c_int, [ctypes.c_int, vp, ctypes.c_size_t, u32p]),
    ("mck_builtin_checksum_with_last_byte_r", ctypes.c_int,
     [ctypes.c_int, vp, ctypes.c_size_t, ctypes.c_char, u32p]),
    ("mck_np_hash64_r", ctypes.c_int, [vp, ctypes.c_size_t, ctypes.c_uint64, u64p]),
    ("mck_crc32c_batch", ctypes.c_int,
     [ctypes.POINTER(mck_spans), vp, ctypes.c_uint32, vp, vp]),
    ("mck_xxh3_64_batch", ctypes.c_int, [ctypes.POINTER(mck_spans), vp, vp]),
    ("mck_xxh32_batch", ctypes.c_int, [ctypes.POINTER(mck_spans), ctypes.c_uint32, vp, vp]),
    ("mck_xxh64_batch", ctypes.c_int, [ctypes.POINTER(mck_spans), ctypes.c_uint64, vp, vp]),
    ("mck_builtin_checksum_batch", ctypes.c_int,
     [ctypes.c_int, ctypes.POINTER(mck_spans), vp, vp, vp]),
    ("mck_sst_trailer_batch", ctypes.c_int,
     [ctypes.c_int, ctypes.POINTER(mck_spans), vp, vp, ctypes.c_uint32, vp, vp]),
    ("mck_sst_verify_batch", ctypes.c_int,
     [ctypes.c_int, ctypes.POINTER(mck_spans), vp, ctypes.c_uint32, vp, vp, vp, vp, vp]),
    ("mck_wal_record_crc_batch", ctypes.c_int,
     [ctypes.POINTER(mck_spans), vp, ctypes.c_uint32, vp, vp]),
    ("mck_wal_verify_batch", ctypes.c_int,
     [vp, ctypes.c_uint64, ctypes.c_uint32, vp, vp]),
    ("mck_crc32c_long_scratch_words", ctypes.c_uint64, [ctypes.c_uint64]),
    ("mck_crc32c_long", ctypes.c_int,
     [vp, ctypes.c_uint64, ctypes.c_uint32, vp, vp, vp]),
    ("mck_np_hash64", ctypes.c_uint64, [vp, ctypes.c_size_t, ctypes.c_uint64]),
    ("mck_np_hash64_batch", ctypes.c_int, [ctypes.POINTER(mck_spans), ctypes.c_uint64, vp, vp]),
    ("mck_kv_protect_batch", ctypes.c_int,
     [ctypes.c_int, ctypes.POINTER(mck_spans), ctypes.POINTER(mck_spans), vp, vp, vp, vp]),
    ("mck_kv_protect_verify_batch", ctypes.c_int,
     [ctypes.c_int, ctypes.POINTER(mck_spans), ctypes.POINTER(mck_spans), vp, vp, vp,
      ctypes.c_uint32, vp, vp, vp, vp]),
    ("mck_handoff_checksum_batch", ctypes.c_int, [ctypes.POINTER(mck_spans), vp, vp]),
    ("mck_block_kv_scratch_bytes", ctypes.c_uint64, [ctypes.c_uint32]),
    ("mck_block_kv_layout_batch", ctypes.c_int,
     [ctypes.c_int, ctypes.POINTER(mck_spans), vp, vp, vp, vp, vp, vp]),
    ("mck_block_kv_work_bytes", ctypes.c_uint64, [ctypes.c_uint64, ctypes.c_uint64]),
    ("mck_block_kv_protect_batch", ctypes.c_int,
     [ctypes.c_int, ctypes.POINTER(mck_spans), ctypes.c_uint32, vp, vp, vp, ctypes.c_uint64, vp, vp, vp]),
    ("mck_block_kv_verify_batch", ctypes.c_int,
     [ctypes.c_int, ctypes.POINTER(mck_spans), ctypes.c_uint32, vp, vp, vp, ctypes.c_uint64, vp, vp, vp,
      vp, vp]),
    ("mck_block_kv_blocks_work_bytes", ctypes.c_uint64, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]),
    ("mck_block_kv_protect_blocks_batch", ctypes.c_int,
     [ctypes.c_int, ctypes.POINTER(mck_spans), ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, vp, vp, vp, vp,
      vp, vp, vp]),
    ("mck_block_kv_verify_blocks_batch", ctypes.c_int,
     [ctypes.c_int, ctypes.POINTER(mck_spans), ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, vp,
      ctypes.c_uint64, vp, vp, vp, vp, vp, vp, vp]),
    ("mck_sst_decode_footer", ctypes.c_int, [vp, ctypes.c_uint64, ctypes.c_uint64, vp]),
    ("mck_sst_list_blocks", ctypes.c_int, [vp, ctypes.c_uint64, vp, vp, ctypes.c_uint64, vp]),
    ("mck_sst_list_blocks_uncompress", ctypes.c_int, [vp, ctypes.c_uint64, vp, vp, vp, vp, ctypes.c_uint64, vp]),
    ("mck_sst_index_handles", ctypes.c_int, [vp, ctypes.c_uint64, ctypes.c_int, ctypes.c_uint32, ctypes.c_int, vp,
                                             ctypes.c_uint64, vp]),
    ("mck_sst_verify_footer", ctypes.c_int, [vp, vp]),
    ("mck_wal_plan", ctypes.c_int,
     [vp, vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, vp, ctypes.c_uint64, vp, vp, vp]),
    ("mck_wal_write_batch", ctypes.c_int,
     [vp, vp, ctypes.c_uint32, ctypes.c_uint32, vp, vp, vp]),
    ("mck_wal_list_records", ctypes.c_int,
     [vp, ctypes.c_uint64, ctypes.c_uint32, vp, ctypes.c_uint64, vp, vp, vp, ctypes.c_uint64, vp, vp]),
    ("mck_wal_gather_batch", ctypes.c_int, [vp, vp, ctypes.c_uint32, vp, vp]),
    ("mck_wal_read_records", ctypes.c_int, [vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, vp, vp]),
    ("mck_wal_reason_string", ctypes.c_char_p, [ctypes.c_int]),
    ("mck_wal_recover_batch", ctypes.c_int, [vp, vp, ctypes.c_uint32, ctypes.c_uint32, vp, vp, vp]),
    ("mck_wal_plan_records", ctypes.c_int, [vp, ctypes.c_uint64, ctypes.c_uint32, vp, ctypes.c_uint64, vp]),
    ("mck_wal_recover", ctypes.c_int,
     [vp, vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, vp, vp]),
    ("mck_wal_recovery_read_out", ctypes.c_int, [vp, vp]),
    ("mck_wal_recovery_checksums", ctypes.c_int, [vp, vp, ctypes.c_uint64]),
    ("mck_wal_recovery_get_info", ctypes.c_int, [vp, vp]),
    ("mck_wal_recovery_block_results", ctypes.c_int, [vp, vp, ctypes.c_uint64]),
    ("mck_wal_recovery_report_positions", ctypes.c_int, [vp, vp, ctypes.c_uint64]),
    ("mck_wal_recovery_free", None, [vp]),
    ("mck_wal_tail_create", ctypes.c_int, [ctypes.c_uint32, vp]),
    ("mck_wal_tail_destroy", None, [vp]),
    ("mck_wal_tail_set_image", ctypes.c_int, [vp, vp, ctypes.c_uint64, vp]),
    ("mck_wal_tail_read_record", ctypes.c_int, [vp, vp, vp, vp]),
    ("mck_wal_tail_record_fragments", ctypes.c_int, [vp, vp, ctypes.c_uint64]),
    ("mck_wal_tail_unmark_eof", ctypes.c_int, [vp]),
    ("mck_wal_tail_is_eof", ctypes.c_int, [vp]),
    ("mck_wal_tail_old_record", ctypes.c_int, [vp, vp]),
    ("mck_wal_tail_pending_verify", ctypes.c_int, [vp, vp, vp]),
    ("mck_wal_tail_add_verdict", ctypes.c_int, [vp, ctypes.c_uint64, vp]),
    ("mck_wal_tail_reports", ctypes.c_int, [vp, vp, ctypes.c_uint64, vp, vp]),
    ("mck_blob_list_records", ctypes.c_int, [vp, ctypes.c_uint64, vp, vp, ctypes.c_uint64, vp]),
    ("mck_blob_record_batch", ctypes.c_int,
     [ctypes.c_int, vp, vp, vp, ctypes.c_uint32, vp, vp, vp]),
    ("mck_partition_spans", ctypes.c_int,
     [vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, vp]),
    ("mck_host_batch_checksum", ctypes.c_int,
     [ctypes.c_int, vp, vp, vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
      ctypes.c_uint32, ctypes.c_int, ctypes.c_size_t, vp, vp,
      ctypes.POINTER(ctypes.c_double)]),
    ("mck_host_pipeline_release", None, []),
    ("mck_statistics_get", ctypes.c_int, [vp, ctypes.c_int]),
    ("mck_test_set_crc_driver", ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    ("mck_test_set_xxh3_driver", ctypes.c_int, [ctypes.c_int]),
    ("mck_test_set_virtual_devices", ctypes.c_int, [ctypes.c_int]),
    ("mck_test_wal_walk_fast", ctypes.c_int, [vp, ctypes.c_uint64, ctypes.c_uint32]),
    ("mck_set_shim_error_policy", ctypes.c_int, [ctypes.c_int, vp, vp]),
    ("mck_test_set_xph3_quads", ctypes.c_int, [ctypes.c_int]),
    ("mck_set_perf_level", ctypes.c_int, [ctypes.c_int]),
    ("mck_get_perf_level", ctypes.c_int, []),
    ("mck_perf_context_get", ctypes.c_int, [vp, ctypes.c_int]),
]

MISSING_SYMBOLS = []
for _name, _res, _args in SIGNATURES:
    try:
        _f = getattr(lib, _name)
    except AttributeError:
        # an older build loaded for an A/B timing run may lack newer entry
        # points (named on stderr); the in-tree library must export every one
        if _OVERRIDE:
            MISSING_SYMBOLS.append(_name)
            continue
        raise
    _f.restype = _res
    _f.argtypes = _args
if MISSING_SYMBOLS:
    print(f"speedb_amd: A/B engine {LIB_PATH} lacks {', '.join(MISSING_SYMBOLS)}", file=sys.stderr)


class MckError(RuntimeError):
    pass


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib.mck_last_error().decode(errors="replace")
        raise MckError(f"{what} failed (rc={rc}): {msg}")

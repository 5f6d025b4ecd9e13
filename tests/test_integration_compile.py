"""The boundary's reference-side adapters (integration/rocksdb_adapters.h,
INTEGRATION.md 2.1 / 2.6) compiled against the reference's OWN headers
(include/rocksdb/file_checksum.h:50-90, table/format.h:119,307-311,
table/block_based/reader_common.h:33-36) with -fsyntax-only: a signature
drift on either side fails here.  Skipped when /root/reference is absent
(the GPU box)."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
HIPCC = "/opt/rocm/bin/hipcc"
pytestmark = pytest.mark.skipif(not (os.path.isdir(os.path.join(REF, "table")) and os.path.exists(HIPCC)),
                                reason="reference tree or hipcc absent")

_TU = """
#include "integration/rocksdb_adapters.h"
namespace A = speedb_amd_rocksdb;
int main() {
  A::GpuFileChecksumGenFactory f;
  ROCKSDB_NAMESPACE::FileChecksumGenContext c;
  auto g = f.CreateFileChecksumGenerator(c);
  ROCKSDB_NAMESPACE::Footer footer;
  std::vector<ROCKSDB_NAMESPACE::BlockHandle> hs;
  std::vector<ROCKSDB_NAMESPACE::Status> st;
  (void)A::VerifyBlockChecksums(footer, nullptr, 0, hs, "f", &st);
  A::UncompressCtx uc{nullptr, 6};
  mck_sst_footer sf{};
  uint64_t n = 0;
  (void)mck_sst_list_blocks_uncompress(nullptr, 0, &A::UncompressWithReference, &uc, &sf, nullptr, 0, &n);
  A::GpuLogRecoveryReader reader(nullptr, 7);
  (void)reader.Recover(nullptr, nullptr, 0, ROCKSDB_NAMESPACE::WALRecoveryMode::kPointInTimeRecovery);
  ROCKSDB_NAMESPACE::Slice rec;
  std::string scratch;
  uint64_t sum = 0;
  (void)reader.ReadRecord(&rec, &scratch, ROCKSDB_NAMESPACE::WALRecoveryMode::kPointInTimeRecovery, &sum);
  std::vector<std::array<char, 5>> tr;
  (void)A::ComputeBlockTrailers(ROCKSDB_NAMESPACE::kCRC32c, 0, nullptr, 0, hs, {}, &tr);
  return g ? 0 : 1;
}
"""


def _compile(tmp_path, header_text=None):
    inc = tmp_path / "inc"
    (inc / "integration").mkdir(parents=True, exist_ok=True)
    src = open(os.path.join(REPO, "integration", "rocksdb_adapters.h")).read()
    (inc / "integration" / "rocksdb_adapters.h").write_text(header_text if header_text is not None else src)
    tu = tmp_path / "tu.cc"
    tu.write_text(_TU)
    cmd = [HIPCC, "-std=c++17", "-fsyntax-only", "-DROCKSDB_PLATFORM_POSIX", "-DROCKSDB_LIB_IO_POSIX",
           "-I", str(inc), "-I", os.path.join(REPO, "include"), "-I", os.path.join(REF, "include"), "-I", REF,
           str(tu)]
    return subprocess.run(cmd, capture_output=True, text=True)


def test_adapters_compile_against_reference_headers(tmp_path):
    r = _compile(tmp_path)
    assert r.returncode == 0, r.stderr[-4000:]


# one drift per pin: the edited header must fail with that pin's message
DRIFTS = [
    ("MCK_WAL_kPointInTimeRecovery &&", "MCK_WAL_kSkipAnyCorruptedRecords &&", "WALRecoveryMode values differ"),
    ("rdb::log::kBlockSize == MCK_WAL_kBlockSize", "rdb::log::kBlockSize == 2 * MCK_WAL_kBlockSize",
     "WAL block / header sizes differ"),
    ("(int)rdb::log::kLastType == speedb_amd::log::kLastType", "(int)rdb::log::kLastType == speedb_amd::log::kMiddleType",
     "WAL record types differ"),
    ("void(size_t, const rdb::Status&)>::value", "void(uint32_t, const rdb::Status&)>::value",
     "Reporter::Corruption signature drifted"),
    ("bool(rdb::Slice*, std::string*, rdb::WALRecoveryMode, uint64_t*)>::value",
     "bool(rdb::Slice*, std::string*, rdb::WALRecoveryMode, uint32_t*)>::value", "ReadRecord signature drifted"),
    ("rdb::BlockBasedTable::kBlockTrailerSize == 5", "rdb::BlockBasedTable::kBlockTrailerSize == 4",
     "block trailer is [type][LE32]"),
]


@pytest.mark.parametrize("old,new,msg", DRIFTS, ids=[d[2].split()[0] + "_" + str(i) for i, d in enumerate(DRIFTS)])
def test_wal_and_trailer_pins_bite(tmp_path, old, new, msg):
    src = open(os.path.join(REPO, "integration", "rocksdb_adapters.h")).read()
    drift = src.replace(old, new, 1)
    assert drift != src, old
    r = _compile(tmp_path, drift)
    assert r.returncode != 0 and msg in r.stderr, r.stderr[-2000:]


def test_signature_drift_fails(tmp_path):
    """The pins bite: the same header expecting a drifted reference signature
    (VerifyBlockChecksum's block_size as uint32_t) does not compile."""
    src = open(os.path.join(REPO, "integration", "rocksdb_adapters.h")).read()
    drift = src.replace("rdb::Status (*)(const rdb::Footer&, const char*, size_t, const std::string&,",
                        "rdb::Status (*)(const rdb::Footer&, const char*, uint32_t, const std::string&,", 1)
    assert drift != src
    r = _compile(tmp_path, drift)
    assert r.returncode != 0 and "signature drifted" in r.stderr

"""The C++ host mirror (include/speedb_amd/checksum.hpp): it compiles against
the C ABI here (CPU), and its restatement of the reference's own gtest cases
(tests/cpp/test_checksum.cc) passes on the GPU."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "tests", "cpp", "test_checksum.cc")
BIN = os.path.join(REPO, "tests", "cpp", "test_checksum")
PKG = os.path.join(REPO, "speedb_amd")


def build():
    if os.path.exists(BIN) and os.path.getmtime(BIN) > max(
            os.path.getmtime(SRC), os.path.getmtime(os.path.join(REPO, "include", "speedb_amd",
                                                                 "checksum.hpp"))):
        return BIN
    cmd = ["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-I", os.path.join(REPO, "include"),
           "-I", os.path.join(REPO, "include", "speedb_amd"), SRC, "-o", BIN,
           "-L", PKG, "-lspeedb_amd", f"-Wl,-rpath,{PKG}"]
    subprocess.check_call(cmd)
    return BIN


def test_cpp_mirror_builds():
    assert os.path.exists(build())


def test_cpp_mirror_fails_loudly_without_a_device():
    """the reference-named functions must not turn a HIP
    error into a checksum of 0 (a re-pointed trailer writer would store it):
    with no GPU visible every one throws DeviceError, and the file checksum
    generator ends kUnknownFileChecksum."""
    env = dict(os.environ, HIP_VISIBLE_DEVICES="-1", ROCR_VISIBLE_DEVICES="-1", CUDA_VISIBLE_DEVICES="-1")
    out = subprocess.run([build(), "--nodevice"], capture_output=True, text=True, timeout=120, env=env)
    print(out.stdout)
    print(out.stderr)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "0 failures" in out.stdout


@pytest.mark.gpu
def test_cpp_mirror_reference_cases(gpu):
    out = subprocess.run([build()], capture_output=True, text=True, timeout=300)
    print(out.stdout)
    print(out.stderr)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "0 failures" in out.stdout


@pytest.mark.gpu
def test_cpp_verify_sst_file(gpu, oracle, tmp_path):
    """speedb_amd::VerifySstFile (C++ mirror of BlockBasedTable::
    VerifyChecksum) on a format_version 6 image from the test writer."""
    from sst_format import write_sst
    img, layout = write_sst(oracle, format_version=6, checksum_type=1, index_type=2, n_data=30,
                            meta=("partitioned_filter", "range_del"))
    path = tmp_path / "000042.sst"
    path.write_bytes(img)
    data = [b for b in layout.blocks if b[2] == "data"]
    bad = data[len(data) // 2][0] + 11
    out = subprocess.run([build(), "--sst", str(path), str(bad)], capture_output=True, text=True, timeout=120)
    print(out.stdout)
    print(out.stderr)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "0 failures" in out.stdout

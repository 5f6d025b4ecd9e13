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


@pytest.mark.gpu
def test_cpp_mirror_reference_cases(gpu):
    out = subprocess.run([build()], capture_output=True, text=True, timeout=300)
    print(out.stdout)
    print(out.stderr)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "0 failures" in out.stdout

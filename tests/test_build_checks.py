"""Build-time checks that run in the container (no GPU): the LDS-image
kernels carry no static LDS (the CRC
table image is addressed from LDS byte 0, so static LDS shifts every table).
"""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import __graft_entry__ as G  # noqa: E402

HIPCC = "/opt/rocm/bin/hipcc"


def test_engine_lds_image_kernels_have_no_static_lds():
    if not os.path.exists(G.LIB):
        pytest.skip("engine not built")
    found = G.check_static_lds(G.LIB)
    for t in G.LDS_IMAGE_KERNELS:
        assert any(t in k for k in found), t
    assert all(v == 0 for v in found.values())


_PROBE = r"""
#include <hip/hip_runtime.h>
namespace mck {
__global__ void k_crc_ragged(int* o, int i) {
  // a private array the compiler promotes to static LDS (what round 4 hit)
  __shared__ int promoted[256];
  promoted[threadIdx.x] = i;
  __syncthreads();
  o[threadIdx.x] = promoted[(threadIdx.x + i) & 255];
}
__global__ void k_wal_write_il(int* o) { o[0] = 2; }
__global__ void k_wal_verify(int* o) { o[0] = 3; }
__global__ void k_wal_recover(int* o) { o[0] = 4; }
}
extern "C" void probe_launch(int* o) { hipLaunchKernelGGL(mck::k_crc_ragged, 1, 256, 0, 0, o, 3); }
"""


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc absent")
def test_static_lds_check_rejects_a_promoted_array(tmp_path):
    """A library in which one LDS-image kernel has static LDS fails the check
    build() runs; the same library without it passes."""
    src = tmp_path / "probe.hip"
    src.write_text(_PROBE)
    so = tmp_path / "probe.so"
    subprocess.check_call([HIPCC, "-O2", "--offload-arch=gfx950", "-fPIC", "-shared", "-o", str(so), str(src)])
    meta = G.kernel_metadata(str(so))
    ragged = [k for k in meta if "k_crc_ragged" in k]
    assert ragged and int(meta[ragged[0]][".group_segment_fixed_size"]) == 1024
    with pytest.raises(RuntimeError, match="static LDS"):
        G.check_static_lds(str(so))
    src.write_text(_PROBE.replace("__shared__ int promoted[256];", "extern __shared__ int promoted[];"))
    subprocess.check_call([HIPCC, "-O2", "--offload-arch=gfx950", "-fPIC", "-shared", "-o", str(so), str(src)])
    assert all(v == 0 for v in G.check_static_lds(str(so)).values())

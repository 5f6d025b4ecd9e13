"""EXPERIMENT (round 5): fine stamps inside the XXH3 wave driver's prologue,
kept in LDS until the end (a global store before a barrier would add its own
write latency to the barrier -- the r5_stamps.py artefact).  Builds
microbench/_variants/stamps_x3.so from a patched copy of speedb_amd/csrc.

  python microbench/r5_stamps_x3.py build | run
"""
import os
import shutil
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "microbench", "_variants", "stamps_x3.so")
NAMES = ["entry", "share", "x3row", "desc", "pfx-b1", "pfx-b2", "pre-b", "short", "first-unit", "end"]

DECL = r"""
__device__ unsigned long long g_x3st[2048][16];
__shared__ unsigned long long s_st[16];  // (only the XXH3 wave kernel uses it)
"""
PATCHES = [
    ("mck_common.hpp", "namespace mck {", "namespace mck {\n" + DECL, 1),
    ("mck_xxh.hpp", "  __shared__ X3Lds s;\n  const uint32_t lane = threadIdx.x & 63, wpb = blockDim.x >> 6, wid = threadIdx.x >> 6;",
     "  __shared__ X3Lds s;\n"
     "#define ST(i) do { if (threadIdx.x == 0) s_st[i] = wall_clock64(); } while (0)\n"
     "  ST(0);\n  const uint32_t lane = threadIdx.x & 63, wpb = blockDim.x >> 6, wid = threadIdx.x >> 6;", 1),
    ("mck_xxh.hpp", "  const uint32_t start = lo, stride = 1, n = hi - lo;",
     "  ST(1);\n  const uint32_t start = lo, stride = 1, n = hi - lo;\n"
     "  asm volatile(\"\" :: \"v\"((uint32_t)X.k0[0]), \"v\"((uint32_t)X.ksw), \"v\"((uint32_t)X.km1)); ST(2);", 1),
    ("mck_xxh.hpp", "    if (threadIdx.x == 0) s.ctr = 0;\n    // pieces per span",
     "    if (threadIdx.x == 0) s.ctr = 0;\n    if (w0 == 0) ST(3);\n    // pieces per span", 1),
    ("mck_xxh.hpp", "      if (lane == 63) s.wsum[wid] = x;\n      __syncthreads();",
     "      if (lane == 63) s.wsum[wid] = x;\n      __syncthreads();\n      if (w0 == 0 && c0 == 0) ST(4);", 1),
    ("mck_xxh.hpp", "      carry += tot;\n      __syncthreads();",
     "      carry += tot;\n      __syncthreads();\n      if (w0 == 0 && c0 == 0) ST(5);", 1),
    ("mck_xxh.hpp", "    if (threadIdx.x == 0) s.pre[wn] = carry;\n    __syncthreads();",
     "    if (threadIdx.x == 0) s.pre[wn] = carry;\n    __syncthreads();\n    if (w0 == 0) ST(6);", 1),
    ("mck_xxh.hpp", "    X3FeedPieces f{&s, wn, wb, stride, 0, base};",
     "    if (w0 == 0) ST(7);\n    X3FeedPieces f{&s, wn, wb, stride, 0, base};", 1),
    ("mck_xxh.hpp", "    x3p_park<PREVIEW>(cur, k0, ke, X, cs);",
     "    x3p_park<PREVIEW>(cur, k0, ke, X, cs);\n    if (threadIdx.x == 0 && s_st[8] == 0) s_st[8] = wall_clock64();", 1),
    ("mck_xxh.hpp", "    xxh3_piece_loop<Op, PREVIEW>(op, f, X);\n  }\n}",
     "    xxh3_piece_loop<Op, PREVIEW>(op, f, X);\n  }\n  __syncthreads();\n  ST(9);\n"
     "  if (threadIdx.x < 10 && blockIdx.x < 2048) g_x3st[blockIdx.x][threadIdx.x] = s_st[threadIdx.x];\n}", 1),
    ("mck_engine.hip", "}  // extern \"C\"",
     "int mck_dbg_x3st(void* host) {\n  return hipMemcpyFromSymbol(host, HIP_SYMBOL(mck::g_x3st), sizeof(mck::g_x3st)) == hipSuccess ? 0 : -2;\n}\n"
     "}  // extern \"C\"", 1),
]


def build():
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "speedb_amd", "csrc")
        shutil.copytree(os.path.join(REPO, "speedb_amd", "csrc"), c)
        shutil.copytree(os.path.join(REPO, "include"), os.path.join(d, "include"))
        for f, a, r, n in PATCHES:
            p = os.path.join(c, f)
            s = open(p).read()
            assert s.count(a) == n, (f, a[:60], s.count(a))
            open(p, "w").write(s.replace(a, r))
        # the first-unit stamp: s_st[8] must start 0
        p = os.path.join(c, "mck_xxh.hpp")
        s = open(p).read()
        s = s.replace("  ST(0);\n", "  if (threadIdx.x < 16) s_st[threadIdx.x] = 0;\n  __syncthreads();\n  ST(0);\n", 1)
        open(p, "w").write(s)
        os.makedirs(os.path.dirname(OUT), exist_ok=True)
        subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC",
                               "-shared", "-o", OUT] +
                              [os.path.join(c, f) for f in ("mck_engine.hip", "mck_sst.cc", "mck_blob.cc",
                                                            "mck_wal.cc")])
    print(OUT)


def run():
    os.environ["SPEEDB_AMD_AB"] = "1"
    os.environ["SPEEDB_AMD_LIB"] = OUT
    sys.path.insert(0, REPO)
    import ctypes
    import numpy as np
    import torch
    import speedb_amd as S
    from speedb_amd import _lib
    from speedb_amd import workloads as W
    f = _lib.lib.mck_dbg_x3st
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p]
    im = W.SstImage(1 << 30, S.ChecksumType.kXXH3, torch.device("cuda", 0), seed=100)
    for _ in range(60):
        im.verify()
    torch.cuda.synchronize()
    im.verify()
    torch.cuda.synchronize()
    buf = np.zeros((2048, 16), dtype=np.uint64)
    assert f(buf.ctypes.data) == 0
    a = buf.astype(np.int64)
    a = a[a[:, 9] > 0]
    t0 = a[:, 0].min()
    pct = lambda x: " ".join(f"{np.percentile(x, q):7.2f}" for q in (0, 10, 50, 90, 100))
    print(f"kXXH3 prologue, {len(a)} workgroups, us since the first entry (p0/10/50/90/100):")
    for i, nm in enumerate(NAMES):
        print(f"  {nm:11s} {pct((a[:, i] - t0) / 100.0)}")
    print("  steps (median of per-workgroup deltas):",
          " ".join(f"{NAMES[i]}={np.median((a[:, i] - a[:, i - 1]) / 100.0):.2f}" for i in range(1, 9)))


if __name__ == "__main__":
    build() if sys.argv[1] == "build" else run()

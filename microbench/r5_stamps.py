"""EXPERIMENT (round 5): per-workgroup s_memrealtime stamps in the SST verify
kernels (k_crc_ragged body/head driver, k_xxh3_wave), built from a PATCHED
COPY of speedb_amd/csrc into microbench/_variants/stamps.so -- the product
sources carry no instrumentation.

  python microbench/r5_stamps.py build           # here (hipcc)
  python microbench/r5_stamps.py run [GiB]       # on the GPU box

Stamps per workgroup (100 MHz): P0 kernel entry, P1 after the prologue
(CRC: table fill; XXH3: share_by_bytes), P2 first window staged (the first
unit is next), P3 driver end (after a barrier), plus the hardware CU id.
"""
import os
import shutil
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "microbench", "_variants", "stamps.so")

STAMP_DECL = r"""
__device__ unsigned long long g_stamps[3][2048][32];
__device__ __forceinline__ void stamp(int k, int p) {
  if (threadIdx.x == 0 && blockIdx.x < 2048) g_stamps[k][blockIdx.x][p] = wall_clock64();
}
__device__ __forceinline__ void stamp_id(int k) {
  if (threadIdx.x == 0 && blockIdx.x < 2048) g_stamps[k][blockIdx.x][k == 2 ? 15 : 4] = __smid();
}
"""

PATCHES = [
    # (file, anchor, replacement)
    ("mck_common.hpp", "namespace mck {", "namespace mck {\n" + STAMP_DECL, 1),
    ("mck_kernels.hpp", "    crc_bh_driver<Op, T>(op, sh, &g_crc_tables);",
     "  { stamp(0, 0); stamp_id(0); crc_bh_driver<Op, T>(op, sh, &g_crc_tables); __syncthreads(); stamp(0, 3); }", 1),
    ("mck_crc_bh.hpp", "  __syncthreads();  // the init tables (read by the staging of empty spans)",
     "  __syncthreads();  // the init tables (read by the staging of empty spans)\n  stamp(0, 1);", 1),
    ("mck_crc_bh.hpp", "    crc_bh_stage(op, sh, w1 - w0, base, kind);",
     "    crc_bh_stage(op, sh, w1 - w0, base, kind);\n    if (wi == 0) stamp(0, 2);", 1),
    ("mck_kernels.hpp", "  xxh3_wave_driver<Op, false>(op, count, 0);",
     "  stamp(1, 0); stamp_id(1); xxh3_wave_driver<Op, false>(op, count, 0); __syncthreads(); stamp(1, 3);", 1),
    ("mck_xxh.hpp", "  const uint32_t start = lo, stride = 1, n = hi - lo;",
     "  stamp(1, 1);\n  const uint32_t start = lo, stride = 1, n = hi - lo;", 1),
    ("mck_xxh.hpp", "    X3FeedPieces f{&s, wn, wb, stride, 0, base};",
     "    if (w0 == 0) stamp(1, 2);\n    X3FeedPieces f{&s, wn, wb, stride, 0, base};", 1),
    ("mck_kernels.hpp", "    crc_rows_windows<Op>(op, sh, lds, &g_crc_tables, force == 8 || force == 9 ? 0 : force);",
     "  { stamp(2, 0); stamp_id(2); crc_rows_windows<Op>(op, sh, lds, &g_crc_tables, force == 8 || force == 9 ? 0 : force);"
     " __syncthreads(); stamp(2, 14); }", 1),
    ("mck_crc.hpp", "    crc_rows_loop<Op, W>(op, sh, g);\n  }",
     "    if (wi < 13) stamp(2, 1 + wi);\n    crc_rows_loop<Op, W>(op, sh, g);\n  }", 1),
    ("mck_crc_bh.hpp", "    *lds_p64(kBLdsAcc + 8 * t) = (uint64_t)(P + hh) << 32;\n  }",
     "    *lds_p64(kBLdsAcc + 8 * t) = (uint64_t)(P + hh) << 32;\n  }\n  if (sh.start == blockIdx.x || true) stamp(0, 5);", 1),
    ("mck_crc_bh.hpp", "  const uint32_t W = bh_head_w((uint32_t)(htot >> 16), (uint32_t)(htot & 0xFFFFu));",
     "  stamp(0, 6);\n  const uint32_t W = bh_head_w((uint32_t)(htot >> 16), (uint32_t)(htot & 0xFFFFu));", 1),
    ("mck_crc_bh.hpp", "  const uint64_t ex = below + x - v;",
     "  stamp(0, 7);\n  const uint64_t ex = below + x - v;", 1),
    ("mck_xxh.hpp", "    if (threadIdx.x == 0) s.ctr = 0;\n    // pieces per span",
     "    if (threadIdx.x == 0) s.ctr = 0;\n    if (w0 == 0) stamp(1, 5);\n    // pieces per span", 1),
    ("mck_xxh.hpp", "    if (threadIdx.x == 0) s.pre[wn] = carry;\n    __syncthreads();",
     "    if (threadIdx.x == 0) s.pre[wn] = carry;\n    if (w0 == 0) stamp(1, 6);\n    __syncthreads();\n    if (w0 == 0) stamp(1, 7);", 1),
    ("mck_crc.hpp", "      __syncthreads();  // every row is done with the previous window's slots\n      row_desc_stage<Op>(op, sh, false);",
     "      __syncthreads();  // every row is done with the previous window's slots\n      if (wi < 13) stamp(2, 16 + wi);\n      row_desc_stage<Op>(op, sh, false);", 1),
    ("mck_engine.hip", "}  // extern \"C\"",
     "int mck_dbg_stamps(void* host) {\n  return hipMemcpyFromSymbol(host, HIP_SYMBOL(mck::g_stamps), sizeof(mck::g_stamps)) == hipSuccess ? 0 : -2;\n}\n"
     "}  // extern \"C\"", 1),
]


def build():
    src = os.path.join(REPO, "speedb_amd", "csrc")
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "speedb_amd", "csrc")
        shutil.copytree(src, c)
        shutil.copytree(os.path.join(REPO, "include"), os.path.join(d, "include"))
        for f, a, r, n in PATCHES:
            p = os.path.join(c, f)
            s = open(p).read()
            assert s.count(a) == n, (f, a, s.count(a))
            open(p, "w").write(s.replace(a, r))
        os.makedirs(os.path.dirname(OUT), exist_ok=True)
        subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC",
                               "-shared", "-o", OUT] +
                              [os.path.join(c, f) for f in ("mck_engine.hip", "mck_sst.cc", "mck_blob.cc",
                                                            "mck_wal.cc")])
    print(OUT)


def run(gib):
    os.environ["SPEEDB_AMD_AB"] = "1"
    os.environ["SPEEDB_AMD_LIB"] = OUT
    sys.path.insert(0, REPO)
    import ctypes
    import numpy as np
    import torch
    import speedb_amd as S
    from speedb_amd import _lib
    from speedb_amd import workloads as W
    dev = torch.device("cuda", 0)
    f = _lib.lib.mck_dbg_stamps
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p]
    for t in (S.ChecksumType.kCRC32c, S.ChecksumType.kXXH3):
        im = W.SstImage(int(gib * (1 << 30)), t, dev, seed=100)
        for _ in range(60):
            im.verify()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        im.verify()
        e1.record()
        torch.cuda.synchronize()
        buf = np.zeros((3, 2048, 32), dtype=np.uint64)
        assert f(buf.ctypes.data) == 0
        k = 0 if t == S.ChecksumType.kCRC32c else 1
        a = buf[k].astype(np.int64)
        a = a[a[:, 3] > 0]
        t0 = a[:, 0].min()
        rel = (a[:, :4] - t0) / 100.0
        pct = lambda x: " ".join(f"{np.percentile(x, q):7.1f}" for q in (0, 10, 50, 90, 100))
        print(f"== {t.name}: {len(a)} workgroups, event time {e0.elapsed_time(e1) * 1e3:.1f} us, "
              f"stamp span {rel[:, 3].max():.1f} us")
        for i, nm in enumerate(("P0 entry", "P1 prologue", "P2 staged", "P3 end")):
            print(f"  {nm:12s} p0/10/50/90/100: {pct(rel[:, i])}")
        print(f"  P1-P0: {pct(rel[:, 1] - rel[:, 0])}   P2-P1: {pct(rel[:, 2] - rel[:, 1])}   "
              f"P3-P2: {pct(rel[:, 3] - rel[:, 2])}")
        fine = (a[:, 5:8] - t0) / 100.0
        for i, nm in enumerate(("S5", "S6", "S7")):
            print(f"  {nm} - P1     : {pct(fine[:, i] - rel[:, 1])}")
        ends = rel[:, 3]
        order = np.argsort(ends)
        print("  slowest 8 (wg, cu id, P2, end):", [(int(i), int(a[i, 4]), round(rel[i, 2], 1), round(ends[i], 1))
                                                   for i in order[-8:]])
        print("  fastest 4:", [(int(i), int(a[i, 4]), round(ends[i], 1)) for i in order[:4]])
        # share bytes of the CRC kernel's count-balanced shares
        if k == 0:
            n = im.count
            G = len(a)
            lens = im.spans.lengths.cpu().numpy().astype(np.int64) if im.spans.lengths is not None else None
            if lens is not None:
                b = np.array([lens[n * g // G:n * (g + 1) // G].sum() for g in range(G)])
                c = np.corrcoef(b, ends[:G])[0, 1]
                print(f"  share bytes p0/50/100: {b.min() / 2**20:.2f} {np.median(b) / 2**20:.2f} "
                      f"{b.max() / 2**20:.2f} MiB; corr(bytes, end) = {c:.3f}")
        del im
        torch.cuda.empty_cache()


def run_rows():
    """The row driver on the WAL-record shape (bench.py --workload walrec):
    per-workgroup window starts."""
    os.environ["SPEEDB_AMD_AB"] = "1"
    os.environ["SPEEDB_AMD_LIB"] = OUT
    sys.path.insert(0, REPO)
    import ctypes
    import numpy as np
    import torch
    import speedb_amd as S
    from speedb_amd import _lib
    from speedb_amd import workloads as W
    dev = torch.device("cuda", 0)
    f = _lib.lib.mck_dbg_stamps
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p]
    rng = np.random.default_rng(800)
    n = int((1 << 30) // 600)
    lens = rng.integers(100, 1101, size=n).astype(np.int64)
    step = lens + 7 + rng.integers(0, 8, size=n)
    offs = np.zeros(n, dtype=np.int64)
    offs[1:] = np.cumsum(step)[:-1]
    data = W.rand_bytes(int(offs[-1] + lens[-1]) + 64, dev, 801)
    sp = S.Spans(data, n, offsets=torch.from_numpy(offs).to(dev), lengths=torch.from_numpy(lens.astype(np.int32)).to(dev))
    types = torch.from_numpy(rng.choice([1, 2, 3, 4], size=n).astype(np.uint8)).to(dev)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    for _ in range(40):
        S.wal_record_crc_batch(sp, types, 7, out=out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    S.wal_record_crc_batch(sp, types, 7, out=out)
    e1.record()
    torch.cuda.synchronize()
    buf = np.zeros((3, 2048, 32), dtype=np.uint64)
    assert f(buf.ctypes.data) == 0
    a = buf[2].astype(np.int64)
    a = a[a[:, 14] > 0]
    t0 = a[:, 0].min()
    pct = lambda x: " ".join(f"{np.percentile(x, q):7.1f}" for q in (0, 10, 50, 90, 100))
    print(f"== walrec rows: {len(a)} workgroups, {n} spans, event {e0.elapsed_time(e1) * 1e3:.1f} us")
    print(f"  entry        : {pct((a[:, 0] - t0) / 100)}")
    for w in range(13):
        col = a[:, 1 + w]
        if (col > 0).sum() < len(a) // 2:
            break
        print(f"  window {w:2d} go: {pct((col[col > 0] - t0) / 100)}")
    print(f"  end          : {pct((a[:, 14] - t0) / 100)}")
    for w in range(1, 13):
        d = a[:, 16 + w]
        g = a[:, 1 + w]
        ok = (d > 0) & (g > 0)
        if ok.sum() < len(a) // 2:
            break
        print(f"  window {w:2d} staging (go - drained): {pct((g[ok] - d[ok]) / 100)}")


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build()
    elif sys.argv[1] == "rows":
        run_rows()
    else:
        run(float(sys.argv[2]) if len(sys.argv) > 2 else 1.0)

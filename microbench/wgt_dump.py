"""EXPERIMENT (variant library microbench/_variants/wgt.so, built with
per-workgroup s_memrealtime stamps in k_crc_ragged / k_xxh3_wave): run one
bench.py command, then print the last launch's workgroup start / end spread.
usage: SPEEDB_AMD_LIB=.../wgt.so python3 microbench/wgt_dump.py <bench args>"""
import atexit
import ctypes
import os
import runpy
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def dump():
    from speedb_amd import _lib
    buf = (ctypes.c_uint64 * (2 * 4096 * 2))()
    if _lib.lib.mck_dbg_wgtimes(buf) != 0:
        print("dump failed")
        return
    a = np.frombuffer(buf, dtype=np.uint64).reshape(2, 4096, 2).astype(np.int64)
    for k, name in enumerate(("k_crc_ragged", "k_xxh3_wave")):
        t = a[k]
        t = t[t[:, 1] > 0]
        if not len(t):
            continue
        t0 = t[:, 0].min()
        st = (t[:, 0] - t0) / 100.0  # us (100 MHz)
        en = (t[:, 1] - t0) / 100.0
        du = en - st
        pc = lambda x: " ".join(f"{v:7.1f}" for v in np.percentile(x, [0, 10, 50, 90, 100]))
        print(f"{name}: {len(t)} workgroups, span {en.max():.1f} us")
        print(f"  start  us  p0/10/50/90/100: {pc(st)}")
        print(f"  end    us  p0/10/50/90/100: {pc(en)}")
        print(f"  length us  p0/10/50/90/100: {pc(du)}")
        idx = np.nonzero(a[k][:, 1] > 0)[0]
        print("  mean end by blockIdx % 8 (XCD):", " ".join(f"{en[idx % 8 == x].mean():6.1f}" for x in range(8)))
        q = len(idx) // 8
        print("  mean end by blockIdx / (G/8):  ", " ".join(f"{en[x * q:(x + 1) * q].mean():6.1f}" for x in range(8)))
        np.save(f"/tmp/wgt_{name}.npy", np.stack([st, en]))
    sys.stdout.flush()


atexit.register(dump)
sys.argv = [os.path.join(REPO, "bench.py")] + sys.argv[1:]
sys.path.insert(0, REPO)
runpy.run_path(os.path.join(REPO, "bench.py"), run_name="__main__")

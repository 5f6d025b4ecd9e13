"""Kernel time of one ragged CRC batch (median of 30, HIP events): the
4/16/64 KiB (+0..255) mix at 1 GiB and 4100-4400-B spans, per driver."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np
import torch
torch.cuda.is_available()
import speedb_amd as S
from speedb_amd import _lib

rng = np.random.default_rng(1)


def mk(sizes, gap):
    offs = np.concatenate([[0], np.cumsum(sizes + gap)[:-1]])
    dev = torch.randint(0, 256, (int(offs[-1] + sizes[-1] + 64),), dtype=torch.uint8, device="cuda")
    return S.Spans(dev, len(sizes), offsets=torch.tensor(offs, device="cuda"),
                   lengths=torch.tensor(sizes.astype(np.int32), device="cuda")), int(sizes.sum())


def timeit(sp):
    for _ in range(5):
        S.crc32c_batch(sp)
    ts = []
    for _ in range(30):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); S.crc32c_batch(sp); b.record(); b.synchronize()
        ts.append(a.elapsed_time(b))
    return float(np.median(ts))


sizes = rng.choice([4096] * 6 + [16384] * 3 + [65536], size=200_000) + rng.integers(0, 256, size=200_000)
sizes = sizes[np.cumsum(sizes + 5) < (1 << 30)]
mix, mixb = mk(sizes, 5)
r41, r41b = mk(rng.integers(4100, 4401, size=250_000).astype(np.int64), 0)
tag = os.environ.get("TAG", "base")
for drv, name in ((0, "auto"), (1, "wave"), (4, "units")):
    _lib.check(_lib.lib.mck_test_set_crc_driver(drv, 0), "drv")
    for wl, sp, nb in (("mix1G", mix, mixb), ("r4100", r41, r41b)):
        ms = timeit(sp)
        print("%s %s %s %.4f ms %.3f of 8 TB/s" % (tag, name, wl, ms, nb / ms / 1e9 / 8.0 ))
_lib.check(_lib.lib.mck_test_set_crc_driver(0, 0), "drv")

"""Row-driver width sweep on the short-span shapes (WAL records 100-1100 B at
byte offsets, 100-300-B spans, 300-700-B spans): the same batch with every
share forced to one row width through the engine's test hook
(mck_test_set_crc_driver: 6 = one lane per span, 5 = 4-lane rows, 3 = 8-lane,
2 = 16-lane, 7 = the body/head driver, 0 = the by-length choice), kernel time from HIP events, best of 20.  Prints one JSON
line per shape: fraction of 8 TB/s per width (same accounting as bench.py:
span bytes + 16 B descriptor/output per span, +1 type byte for WAL records).

  python microbench/rows_width.py [kind:min:max ...]   (kind = walrec | ragged)
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import speedb_amd as S
from speedb_amd import _lib


def batch(kind, lo, hi, total, seed):
    rng = np.random.default_rng(seed)
    n = int(total // ((lo + hi) / 2))
    lens = rng.integers(lo, hi + 1, size=n).astype(np.int64)
    gaps = rng.integers(0, 8, size=n) if kind == "walrec" else np.zeros(n, np.int64)
    step = lens + (7 + gaps if kind == "walrec" else 0)
    offs = np.zeros(n, dtype=np.int64)
    offs[1:] = np.cumsum(step)[:-1]
    data = torch.randint(0, 256, (int(offs[-1] + lens[-1]) + 64,), dtype=torch.uint8, device="cuda")
    sp = S.Spans(data, n, offsets=torch.from_numpy(offs).cuda(), lengths=torch.from_numpy(lens.astype(np.int32)).cuda())
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    if kind == "walrec":
        types = torch.from_numpy(rng.choice([1, 2, 3, 4], size=n).astype(np.uint8)).cuda()
        fn = lambda: S.wal_record_crc_batch(sp, types, 7, out=out)  # noqa: E731
        alg = int(lens.sum()) + n * 17
    else:
        fn = lambda: S.crc32c_batch(sp, out=out)  # noqa: E731
        alg = int(lens.sum()) + n * 16
    return fn, alg, out


def timed(fn):
    for _ in range(10):
        fn()
    best = 1e9
    for _ in range(20):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b))
    return best


def main():
    shapes = [tuple(x.split(":")[0:1]) + tuple(int(v) for v in x.split(":")[1:]) for x in sys.argv[1:]] or [
        ("walrec", 100, 1100), ("ragged", 100, 300), ("ragged", 300, 700), ("ragged", 600, 1100),
        ("walrec", 300, 900), ("ragged", 400, 800), ("ragged", 200, 500)]
    for kind, lo, hi in shapes:
        fn, alg, out = batch(kind, lo, hi, 1 << 30, 7)
        res, ref = {}, None
        import time
        t0 = time.time()
        while time.time() - t0 < 0.4:  # settle the clocks (bench.py --settle-ms)
            fn()
        torch.cuda.synchronize()
        for rep in range(2):  # two passes; the best of each width
            for name, drv in (("auto", 0), ("rows1", 6), ("rows4", 5), ("rows8", 3), ("rows16", 2), ("bh", 7)):
                _lib.check(_lib.lib.mck_test_set_crc_driver(drv, 0), "mck_test_set_crc_driver")
                ms = timed(fn)
                got = out.clone()
                if ref is None:
                    ref = got
                assert torch.equal(got, ref), (kind, name)  # every width, the same CRCs
                res[name] = max(res.get(name, 0), round(alg / (ms * 1e-3) / 8e12, 4))
        _lib.check(_lib.lib.mck_test_set_crc_driver(0, 0), "mck_test_set_crc_driver")
        print(json.dumps({"shape": f"{kind} {lo}-{hi}", "frac": res}))


if __name__ == "__main__":
    main()

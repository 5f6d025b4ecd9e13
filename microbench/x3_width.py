"""XXH3 driver sweep on ragged shapes: the same batch (spans at byte
offsets, back to back with 5-byte gaps like SST blocks) on the wave-per-span
driver and on 16-lane rows, forced through the test hook
mck_test_set_xxh3_driver (1 = wave, 2 = rows); kernel time from HIP events
after a settle phase, best of 20 per pass, two passes.  Prints the fraction
of 8 TB/s (span bytes + 16 B descriptor/output per span) per driver.

  python microbench/x3_width.py [min:max | u:len ...]
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import speedb_amd as S  # noqa: E402
from speedb_amd import _lib  # noqa: E402


def main():
    # "min:max" = ragged spans; "u:len" = a uniform batch (stride = length)
    shapes = [tuple(x.split(":")) for x in sys.argv[1:]] or [
        ("500", "1500"), ("1000", "3000"), ("2000", "4000"), ("3000", "5000"), ("4096", "4351"), ("8000", "16000")]
    for a, b in shapes:
        if a == "u":
            L = int(b)
            n = (1 << 30) // L
            lens = np.full(n, L, dtype=np.int64)
            data = torch.randint(0, 256, (n * L + 64,), dtype=torch.uint8, device="cuda")
            sp = S.Spans(data, n, stride=L, length=L)
            lo = hi = L
        else:
            lo, hi = int(a), int(b)
            rng = np.random.default_rng(lo + hi)
            n = int((1 << 30) // ((lo + hi) / 2))
            lens = rng.integers(lo, hi + 1, size=n).astype(np.int64)
            offs = np.zeros(n, dtype=np.int64)
            offs[1:] = np.cumsum(lens + 5)[:-1]
            data = torch.randint(0, 256, (int(offs[-1] + lens[-1]) + 64,), dtype=torch.uint8, device="cuda")
            sp = S.Spans(data, n, offsets=torch.from_numpy(offs).cuda(),
                         lengths=torch.from_numpy(lens.astype(np.int32)).cuda())
        out = torch.empty(n, dtype=torch.int64, device="cuda")
        fn = lambda: S.xxh3_64_batch(sp, out=out)  # noqa: E731
        alg = int(lens.sum()) + n * 16
        t0 = time.time()
        while time.time() - t0 < 0.4:
            fn()
        torch.cuda.synchronize()
        res, ref = {}, None
        for _ in range(2):
            for name, drv in (("wave", 1), ("rows", 2)):
                _lib.check(_lib.lib.mck_test_set_xxh3_driver(drv), "mck_test_set_xxh3_driver")
                for _ in range(5):
                    fn()
                best = 1e9
                for _ in range(20):
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record()
                    fn()
                    b.record()
                    b.synchronize()
                    best = min(best, a.elapsed_time(b))
                got = out.clone()
                ref = got if ref is None else ref
                assert torch.equal(got, ref), name
                res[name] = max(res.get(name, 0), round(alg / (best * 1e-3) / 8e12, 4))
        _lib.check(_lib.lib.mck_test_set_xxh3_driver(0), "mck_test_set_xxh3_driver")
        print(json.dumps({"shape": f"uniform {lo}" if a == "u" else f"{lo}-{hi}", "frac": res}))


if __name__ == "__main__":
    main()

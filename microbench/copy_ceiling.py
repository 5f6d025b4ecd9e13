"""Read+write ceiling on this box: device-to-device copies of the WAL
writer's stream size (2.22 GB), torch copy_ and hipMemcpyAsync D2D, best of
10, reported as (read + write bytes) / time against the 8 TB/s HBM peak --
the same accounting as bench.py's walwrite roofline."""
import json
import torch

n = 2217106570
src = torch.randint(0, 255, (n,), dtype=torch.uint8, device="cuda")
dst = torch.empty_like(src)
s4 = src[: n // 16 * 16].view(torch.int32)
d4 = dst[: n // 16 * 16].view(torch.int32)
res = {}
for name, f in [("torch_copy_u8", lambda: dst.copy_(src)), ("torch_copy_i32", lambda: d4.copy_(s4))]:
    for _ in range(3):
        f()
    best = 1e9
    for _ in range(10):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        f()
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b))
    res[name] = {"ms": round(best, 4), "frac_of_8TBs": round(2 * n / (best * 1e-3) / 8e12, 4)}
print(json.dumps(res))

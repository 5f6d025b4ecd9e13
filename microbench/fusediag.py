"""Generic CRC batch vs oracle for full-round + head-mini-round spans (design diagnostic)."""
import ctypes, os, sys
import numpy as np
import torch
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import speedb_amd as S
ol = ctypes.CDLL(os.path.join(R, "oracle", "liboracle.so"))
ol.orc_crc32c_value.restype = ctypes.c_uint32
ol.orc_crc32c_value.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
rng = np.random.default_rng(5)
N = (int(sys.argv[1]) if len(sys.argv) > 1 else 64) << 20
host = rng.integers(0, 256, N, dtype=np.uint8).tobytes()
dev = torch.frombuffer(bytearray(host), dtype=torch.uint8).cuda()
cases = [(62, 4112, 4144, 12000), (62, 4112, 4144, 64), (3, 4097, 4101, 5000),
         (0, 4100, 4100, 5000), (5, 8200, 8205, 3000), (7, 5000, 5001, 4000)]
if len(sys.argv) > 1:  # many spans: the static feed (share > the LDS descriptor cache)
    cases = [(62, 4112, 4144, (N - 4096) // 4144), (7, 5000, 5001, (N - 8192) // 5001),
             (0, 1000, 1008, 450000)]
for start, length, stride, count in cases:
    offs = [start + stride * i for i in range(count)]
    o = torch.tensor(offs, dtype=torch.int64, device="cuda")
    l_ = torch.full((count,), length, dtype=torch.int32, device="cuda")
    got = S.crc32c_batch(S.Spans(dev, count, offsets=o, lengths=l_)).cpu().numpy().view(np.uint32)
    idx = range(count) if count <= 20000 else list(range(0, 8192)) + list(range(8192, count, 97))
    bad = [i for i in idx if int(got[i]) != ol.orc_crc32c_value(host[offs[i]:offs[i] + length], length)]
    print(start, length, stride, count, "bad", len(bad), bad[:8])

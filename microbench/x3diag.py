"""XXH3 batch diagnostic: which (start offset, length) cells disagree with the oracle."""
import ctypes, os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import speedb_amd as S
ol = ctypes.CDLL(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "liboracle.so"))
ol.orc_xxh3_64.restype = ctypes.c_uint64
ol.orc_xxh3_64.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
rng = np.random.default_rng(1)
host = rng.integers(0, 256, 1 << 20, dtype=np.uint8).tobytes()
dev = torch.frombuffer(bytearray(host), dtype=torch.uint8).cuda()
lens = [241, 255, 256, 257, 300, 1000, 1023, 1024, 1025, 1088, 2048, 4095, 4096, 4097, 5000, 17000]
for mode in ["ragged", "uniform"]:
    bad = []
    for sh in range(8):
        for n in lens:
            if mode == "ragged":
                offs = [sh + 20000 * i for i in range(3)]
                o = torch.tensor(offs, dtype=torch.int64, device="cuda")
                l_ = torch.tensor([n] * 3, dtype=torch.int32, device="cuda")
                sp = S.Spans(dev, 3, offsets=o, lengths=l_)
            else:
                offs = [sh + 20000 * i for i in range(3)]
                sp = S.Spans(dev[sh:], 3, stride=20000, length=n)
            got = [int(x) & (2**64 - 1) for x in S.xxh3_64_batch(sp).cpu().tolist()]
            want = [ol.orc_xxh3_64(host[off:off + n], n) for off in offs]
            if got != want:
                bad.append((sh, n, sum(g != w for g, w in zip(got, want))))
    print(mode, "bad cells:", bad if bad else "none")

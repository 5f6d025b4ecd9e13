"""Blob-record CRC write/verify vs the oracle (design diagnostic): bench-shaped image."""
import ctypes, os, sys
import numpy as np
import torch
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import speedb_amd as S
from speedb_amd import workloads as W
ol = ctypes.CDLL(os.path.join(R, "oracle", "liboracle.so"))
ol.orc_crc32c_value.restype = ctypes.c_uint32
ol.orc_crc32c_value.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
mask = lambda c: ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + 0xa282ead8) & 0xFFFFFFFF
dev = torch.device("cuda", 0)
n, kb = int(sys.argv[1]) if len(sys.argv) > 1 else 200000, 16
vb = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
rec = 32 + kb + vb
img = W.rand_bytes(30 + n * rec + 64, dev, 700)
recs = img[30:30 + n * rec].view(n, rec)
recs[:, 0:8] = torch.tensor(list(kb.to_bytes(8, "little")), dtype=torch.uint8, device=dev)
recs[:, 8:16] = torch.tensor(list(vb.to_bytes(8, "little")), dtype=torch.uint8, device=dev)
offs = 30 + torch.arange(n, dtype=torch.int64, device=dev) * rec
lens = torch.full((n,), kb + vb, dtype=torch.int32, device=dev)
S.blob.WriteRecordCrcs(img, offs, lens)
torch.cuda.synchronize()
h = img.cpu().numpy().tobytes()
badw = []
for i in list(range(0, n, max(1, n // 2000))) + [n - 1]:
    o = 30 + i * rec
    hc = mask(ol.orc_crc32c_value(h[o:o + 24], 24))
    bc = mask(ol.orc_crc32c_value(h[o + 32:o + rec], kb + vb))
    sh, sb = int.from_bytes(h[o + 24:o + 28], "little"), int.from_bytes(h[o + 28:o + 32], "little")
    if hc != sh or bc != sb:
        badw.append((i, hc != sh, bc != sb))
print("write: sampled bad", len(badw), badw[:6])
st = S.blob.record_batch(False, img, offs, lens)
torch.cuda.synchronize()
s = st.cpu().numpy()
bad = np.nonzero(s)[0]
print("verify: bad", len(bad), bad[:8].tolist(), np.bincount(s, minlength=4).tolist())

"""Synthetic, device-resident workloads in the reference's on-disk layouts,
for the benchmark configs of BASELINE.json.  Everything is generated on the
GPU with torch (random bytes) and the engine's own write-side kernels (block
trailers, WAL record headers), so the images are exactly what a Speedb
writer would have produced for those payloads.

* ``uniform_blocks``  -- configs[1]: N x B random blocks, back to back.
* ``sst_image``       -- configs[2]: compaction-shaped run of data blocks,
  4/16/64 KiB at 60/30/10 % plus 0..255 B jitter, each followed by its
  5-byte trailer [compression type][LE32 checksum + context modifier]
  (block_based_table_builder.cc:1304-1358), format_version 6 context
  checksums (random base_context_checksum, real file offsets).
* ``wal_image``       -- configs[3]: 32 KiB WAL blocks, each holding one
  kFullType record with a 32761-byte payload (log_writer.cc:79-175).
"""
from __future__ import annotations

import numpy as np
import torch

from . import checksum as C


def rand_bytes(n: int, device, seed: int):
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    return torch.randint(0, 256, (n,), dtype=torch.uint8, device=device, generator=g)


def uniform_blocks(count: int, block: int, device, seed: int = 1000):
    data = rand_bytes(count * block + 64, device, seed)
    return data, C.Spans.uniform(data, block, count)


class SstImage:
    """A run of block-based-table data blocks in device memory."""

    def __init__(self, total_bytes: int, checksum_type: int, device, seed: int = 7,
                 base_context_checksum: int = 0x5EED1234, file_start: int = 4096):
        rng = np.random.default_rng(seed)
        sizes = []
        acc = 0
        while acc < total_bytes:
            n = int(rng.choice([4096, 16384, 65536], p=[0.6, 0.3, 0.1]) + rng.integers(0, 256))
            sizes.append(n)
            acc += n + 5
        sizes = np.array(sizes, dtype=np.int64)
        offs = np.zeros(len(sizes), dtype=np.int64)
        offs[1:] = np.cumsum(sizes + 5)[:-1]
        self.count = len(sizes)
        self.payload_bytes = int(sizes.sum())
        self.nbytes = int(offs[-1] + sizes[-1] + 5)
        self.checksum_type = int(checksum_type)
        self.base_context_checksum = base_context_checksum
        self.data = rand_bytes(self.nbytes + 64, device, seed)
        self.offsets = torch.from_numpy(offs).to(device)
        self.lengths = torch.from_numpy(sizes.astype(np.int32)).to(device)
        self.file_offsets = self.offsets + file_start
        comp = torch.from_numpy(rng.choice([0, 1, 7], size=self.count).astype(np.uint8)).to(device)
        self.spans = C.Spans(self.data, self.count, offsets=self.offsets, lengths=self.lengths)
        # write side: trailer checksums for every block, then scatter the
        # 5-byte trailers [type][LE32] behind the payloads
        ck = C.sst_trailer_batch(self.checksum_type, self.spans, comp, file_offsets=self.file_offsets,
                                 base_context_checksum=base_context_checksum)
        trailer = torch.empty((self.count, 5), dtype=torch.uint8, device=device)
        trailer[:, 0] = comp
        trailer[:, 1:] = ck.view(torch.uint8).view(self.count, 4)
        pos = (self.offsets + self.lengths.to(torch.int64)).unsqueeze(1) + torch.arange(5, device=device)
        self.data[pos.reshape(-1)] = trailer.reshape(-1)
        torch.cuda.synchronize(device)
        self.outs = (torch.empty(self.count, dtype=torch.uint8, device=device), None, None)

    def verify(self, stream=None, with_count=False):
        """VerifyBlockChecksum of every block into preallocated outputs;
        returns (mismatch, computed, stored, mismatch_count)."""
        return C.sst_verify_batch(self.checksum_type, self.spans, file_offsets=self.file_offsets,
                                  base_context_checksum=self.base_context_checksum, stream=stream,
                                  outs=self.outs, with_count=with_count)

    def corrupt(self, idx):
        """Flip one payload byte in each listed block."""
        for i in idx:
            p = int(self.offsets[i]) + 17
            self.data[p] ^= 0x20


class WalImage:
    """nblocks x 32 KiB WAL blocks, each one kFullType record (payload
    32761 B); its record CRCs come from the write-side kernel."""

    PAYLOAD = 32768 - 7

    def __init__(self, nblocks: int, device, seed: int = 11, log_number: int = 7):
        self.nblocks = nblocks
        self.nbytes = nblocks * 32768
        self.log_number = log_number
        self.data = rand_bytes(self.nbytes + 64, device, seed)
        blocks = self.data[:self.nbytes].view(nblocks, 32768)
        pay = C.Spans(self.data, nblocks, stride=32768, length=self.PAYLOAD)
        pay.base = self.data[7:]  # payload of block b starts at b*32768 + 7
        types = torch.ones(nblocks, dtype=torch.uint8, device=device)  # kFullType
        crc = C.wal_record_crc_batch(pay, types, log_number)
        blocks[:, 0:4] = crc.view(torch.uint8).view(nblocks, 4)
        blocks[:, 4] = self.PAYLOAD & 0xFF
        blocks[:, 5] = self.PAYLOAD >> 8
        blocks[:, 6] = 1
        torch.cuda.synchronize(device)
        self.results = torch.empty((nblocks, 4), dtype=torch.int32, device=device)

    def verify(self, stream=None):
        return C.wal_verify_batch(self.data, self.nbytes, self.log_number, stream=stream,
                                  out=self.results)


def _varint(v: int) -> bytes:
    out = bytearray()
    while v >= 128:
        out.append((v & 127) | 128)
        v >>= 7
    out.append(v)
    return bytes(out)


class DataBlocks:
    """Row 8f-4: uncompressed data blocks as BlockBuilder lays them out
    (table/block_based/block_builder.cc:188-252: prefix-compressed internal
    keys, restart every ``restart_interval`` entries, restart array + footer),
    cut at ``block_bytes`` like FlushBlockBySizePolicy, back to back with a
    5-byte trailer gap between blocks as in an SST.  ``distinct`` different
    blocks are built on the host and tiled to ``count`` blocks on the device
    (throughput does not depend on the bytes repeating: 4 GiB >> L2/MALL).
    ``entries[j]`` keeps block j's (internal key, value) list for checks."""

    def __init__(self, count: int, device, key_bytes: int = 16, value_bytes: int = 1000,
                 block_bytes: int = 4096, restart_interval: int = 16, distinct: int = 256, seed: int = 3):
        rng = np.random.default_rng(seed)
        self.entries, blobs = [], []
        uk = 0
        for _ in range(distinct):
            ents, size = [], 0
            while size < block_bytes:
                user = b"%0*d" % (key_bytes, uk)
                uk += int(rng.integers(1, 50))
                ikey = user + int((int(rng.integers(1, 1 << 56)) << 8) | 1).to_bytes(8, "little")
                val = rng.integers(0, 256, size=value_bytes, dtype=np.uint8).tobytes()
                ents.append((ikey, val))
                size += len(ikey) + len(val) + 3
            self.entries.append(ents)
            buf, restarts, last = bytearray(), [], b""
            for i, (k, v) in enumerate(ents):
                if i % restart_interval == 0:
                    restarts.append(len(buf))
                    sh = 0
                else:
                    sh = 0
                    while sh < min(len(k), len(last)) and k[sh] == last[sh]:
                        sh += 1
                buf += _varint(sh) + _varint(len(k) - sh) + _varint(len(v)) + k[sh:] + v
                last = k
            for r in restarts:
                buf += int(r).to_bytes(4, "little")
            buf += len(restarts).to_bytes(4, "little")
            blobs.append(bytes(buf))
        lens = np.array([len(b) for b in blobs], dtype=np.int64)
        tile_offs = np.zeros(distinct, dtype=np.int64)
        tile_offs[1:] = np.cumsum(lens + 5)[:-1]
        tile_bytes = int(tile_offs[-1] + lens[-1] + 5)
        tile = np.zeros(tile_bytes, dtype=np.uint8)
        for o, b in zip(tile_offs, blobs):
            tile[o:o + len(b)] = np.frombuffer(b, dtype=np.uint8)
        reps = (count + distinct - 1) // distinct
        self.count = count
        self.distinct = distinct
        self.nbytes = reps * tile_bytes
        self.data = torch.empty(self.nbytes + 64, dtype=torch.uint8, device=device)
        self.data[:self.nbytes].view(reps, tile_bytes).copy_(
            torch.from_numpy(tile).to(device).unsqueeze(0).expand(reps, tile_bytes))
        j = np.arange(count) % distinct
        offs = (np.arange(count) // distinct) * tile_bytes + tile_offs[j]
        self.block_lengths = lens[j]
        self.offsets = torch.from_numpy(offs).to(device)
        self.lengths = torch.from_numpy(self.block_lengths.astype(np.int32)).to(device)
        self.block_bytes = int(self.block_lengths.sum())
        self.keys_per_block = np.array([len(e) for e in self.entries])[j]
        self.spans = C.Spans(self.data, count, offsets=self.offsets, lengths=self.lengths)
        torch.cuda.synchronize(device)

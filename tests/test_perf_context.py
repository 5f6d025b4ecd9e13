"""PerfContext::block_checksum_time (include/rocksdb/perf_context.h:97): the
reference times every VerifyBlockChecksum (table/block_based/reader_common.cc
:29, PERF_TIMER_GUARD) into the calling thread's perf context when the
PerfLevel allows (include/rocksdb/perf_level.h).  Here a verify batch's
DEVICE time is measured by an event pair on its stream and attributed to the
thread that issued it."""
import threading

import pytest

from formats import sst_blocks, splitmix_bytes


def test_perf_level_api():
    import speedb_amd as S
    assert S.GetPerfLevel() == S.PerfLevel.kEnableCount  # the reference's default
    S.SetPerfLevel(S.PerfLevel.kEnableTime)
    assert S.GetPerfLevel() == S.PerfLevel.kEnableTime
    with pytest.raises(S.MckError if hasattr(S, "MckError") else Exception):
        S.SetPerfLevel(0)
    S.SetPerfLevel(S.PerfLevel.kEnableCount)
    ctx = S.get_perf_context(reset=True)
    assert set(ctx) == {"block_checksum_time", "block_checksum_count", "block_checksum_batches"}
    # per thread: another thread starts at the default level
    seen = []
    t = threading.Thread(target=lambda: seen.append(S.GetPerfLevel()))
    S.SetPerfLevel(S.PerfLevel.kDisable)
    t.start()
    t.join()
    assert seen == [S.PerfLevel.kEnableCount]
    S.SetPerfLevel(S.PerfLevel.kEnableCount)


@pytest.mark.gpu
def test_block_checksum_time(gpu, oracle):
    import speedb_amd as S
    torch = gpu
    sizes = [4096 + (i * 37) % 256 for i in range(4000)]
    payloads = [splitmix_bytes(7 + i, n) for i, n in enumerate(sizes)]
    img, offs, lens = sst_blocks(oracle, payloads, 1, [0] * len(sizes), 0, 0)
    dev = torch.frombuffer(bytearray(img + bytes(64)), dtype=torch.uint8).to("cuda")
    sp = S.Spans(dev, len(sizes), offsets=torch.tensor(offs, dtype=torch.int64, device="cuda"),
                 lengths=torch.tensor(lens, dtype=torch.int32, device="cuda"))
    S.get_perf_context(reset=True)
    # kEnableCount: counts, no time
    S.sst_verify_batch(1, sp)
    ctx = S.get_perf_context(reset=True)
    assert ctx["block_checksum_count"] == len(sizes) and ctx["block_checksum_batches"] == 1
    assert ctx["block_checksum_time"] == 0
    # a timing level: device time of every batch, read after they complete
    S.SetPerfLevel(S.PerfLevel.kEnableTimeExceptForMutex)
    try:
        for _ in range(3):
            mm, _, _, cnt = S.sst_verify_batch(1, sp)
        ctx = S.get_perf_context(reset=True)
        assert int(cnt.item()) == 0
        assert ctx["block_checksum_count"] == 3 * len(sizes) and ctx["block_checksum_batches"] == 3
        assert ctx["block_checksum_time"] > 0
        # the time is the kernels', not the host's: well under a second here
        assert ctx["block_checksum_time"] < 1e9
        # kDisable: nothing
        S.SetPerfLevel(S.PerfLevel.kDisable)
        S.sst_verify_batch(1, sp)
        ctx = S.get_perf_context()
        assert ctx == {"block_checksum_time": 0, "block_checksum_count": 0, "block_checksum_batches": 0}
    finally:
        S.SetPerfLevel(S.PerfLevel.kEnableCount)

"""The ragged-batch CRC drivers against the oracle.  A ragged batch is one
launch of k_crc_ragged; each workgroup runs its share on the row drivers
(one lane, 4-, 8- or 16-lane rows per span, mck_crc.hpp crc_rows_loop, for
shares of short spans) or the body/head driver (mck_crc_bh.hpp, the rest).
Every
driver is also forced for every workgroup in a child process over the
generic-op parity tests (mck_test_set_crc_driver, set by tests/conftest.py
from SPEEDB_AMD_TEST_CRC_DRIVER / _ORDER)."""
import os
import random
import subprocess
import sys

import numpy as np
import pytest

from formats import splitmix_bytes

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _batch(torch, seed, lens, gap=64):
    rnd = random.Random(seed)
    offs, pos = [], 0
    for n in lens:
        pos += rnd.randrange(0, gap)
        offs.append(pos)
        pos += n
    host = splitmix_bytes(seed, pos + 64)
    dev = torch.frombuffer(bytearray(host), dtype=torch.uint8).to("cuda")
    return host, dev, offs


def test_wal_record_crc_small_ragged_many(gpu, oracle):
    """100K WAL records of 0..1100 B at every alignment: far more spans than
    rows (each row walks ~6 spans), records crossing 1 KiB rounds."""
    import speedb_amd as S
    torch = gpu
    rnd = random.Random(17)
    lens = [rnd.randrange(0, 1101) for _ in range(100_000)]
    lens[:40] = list(range(0, 40))
    host, dev, offs = _batch(torch, 17, lens)
    types = [rnd.choice([1, 2, 3, 4, 5, 6, 7, 8]) for _ in lens]
    sp = S.Spans(dev, len(lens), offsets=torch.tensor(offs, dtype=torch.int64, device="cuda"),
                 lengths=torch.tensor(lens, dtype=torch.int32, device="cuda"))
    got = S.wal_record_crc_batch(sp, torch.tensor(types, dtype=torch.uint8, device="cuda"), 0xC0FFEE)
    got = got.cpu().numpy().view(np.uint32)
    for k in range(len(lens)):
        o, n, t = offs[k], lens[k], types[k]
        assert int(got[k]) == oracle.WalRecordCrc(t, host[o:o + n], t >= 5, 0xC0FFEE), (k, n, t)


def _forced(env):
    """Run the generic CRC parity tests in a child pytest whose conftest sets
    the engine's test hook (mck_test_set_crc_driver) from env."""
    tests = [os.path.join(HERE, "test_crc_rows.py") + "::test_wal_record_crc_small_ragged_many"]
    tests += [os.path.join(HERE, "test_gpu_parity.py") + "::" + t for t in (
        "test_crc32c_batch_ragged", "test_sst_trailer_and_verify", "test_empty_and_zero_inputs",
        "test_large_ragged_batches_static_and_dynamic_feeds", "test_wal_record_crc_batch",
        "test_crc32c_known_answers_on_device", "test_builtin_checksum_batch", "test_sst_verify_large_static_feed",
        "test_checksum_schemas_on_device", "test_scalar_shims", "test_crc32c_long_vs_oracle")]
    tests += [os.path.join(HERE, "test_blob_file.py"), os.path.join(HERE, "test_sst_file.py"),
              os.path.join(HERE, "test_crc_long.py")]
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-m", "gpu", "-p", "no:cacheprovider",
                        "-k", "not subprocess"] + tests,
                       env=dict(os.environ, **env), cwd=os.path.dirname(HERE), capture_output=True, text=True,
                       timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert " passed" in r.stdout


@pytest.mark.parametrize("mode", ["rows16", "rows8", "rows4", "rows1", "bh", "small", "interleaved", "x3rows",
                                  "x3wave"])
def test_auto_kernel_forced_drivers_subprocess(gpu, mode):
    """k_crc_ragged with each driver forced for every workgroup (its choice is
    by mean length, so a parity test of mixed lengths may exercise only one):
    short spans, 0-byte spans, WAL / blob / SST ops on every driver; and the
    interleaved span order instead of contiguous ranges.  "small": the
    wave-per-span path for every share it accepts (<= 16 spans of <= 16 KiB),
    in batches of any size -- by default only batches of <= 64 spans.
    "x3rows" / "x3wave": every XXH3 batch (ragged or uniform) on the 16-lane
    rows kernel / the wave kernel (which itself takes rows for shares of
    256 B - 2.5 KiB spans)."""
    if (os.environ.get("SPEEDB_AMD_TEST_CRC_DRIVER") or os.environ.get("SPEEDB_AMD_TEST_CRC_ORDER")
            or os.environ.get("SPEEDB_AMD_TEST_X3_DRIVER")):
        pytest.skip("already running a forced driver")
    _forced({"SPEEDB_AMD_TEST_CRC_ORDER": "interleaved"} if mode == "interleaved"
            else {"SPEEDB_AMD_TEST_X3_DRIVER": mode[2:]} if mode.startswith("x3")
            else {"SPEEDB_AMD_TEST_CRC_DRIVER": mode})

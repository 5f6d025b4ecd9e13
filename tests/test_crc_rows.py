"""The ragged-batch CRC drivers against the oracle.  By default a ragged
batch runs on k_crc_auto, which picks per workgroup (from its share's mean
span length) the row driver with 8- or 16-lane rows (one row per span,
mck_crc.hpp crc_rows_loop) or the wave driver (crc_drive).  Every driver is
also forced in a child process over the generic-op parity tests (the A/B
switches are read once per process): MCK_CRC_AUTO=wave|rows16|rows8 inside
the auto kernel, MCK_CRC_ROWS=1 (+ MCK_CRC_ROW_LANES) for the standalone row
kernel, MCK_CRC_ROWS=0 for the standalone wave kernel with its static feed."""
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


def test_generic_ops_through_rows_subprocess(gpu):
    """CRC value/extend/mask, SST trailer + verify (context checksums,
    corruption), blob records and WAL paths with MCK_CRC_ROWS=1."""
    if os.environ.get("MCK_CRC_ROWS") or os.environ.get("MCK_CRC_AUTO"):
        pytest.skip("already running a forced driver")
    env = dict(os.environ, MCK_CRC_ROWS="1")
    tests = [os.path.join(HERE, "test_gpu_parity.py") + "::" + t for t in (
        "test_crc32c_batch_ragged", "test_crc32c_known_answers_on_device", "test_scalar_shims",
        "test_checksum_schemas_on_device", "test_builtin_checksum_batch", "test_sst_trailer_and_verify",
        "test_wal_record_crc_batch", "test_wal_verify_batch", "test_empty_and_zero_inputs",
        "test_large_ragged_batches_static_and_dynamic_feeds", "test_crc32c_long_vs_oracle",
        "test_sst_verify_large_static_feed")]
    tests += [os.path.join(HERE, "test_blob_file.py"), os.path.join(HERE, "test_sst_file.py")]
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-m", "gpu", "-p", "no:cacheprovider"] + tests,
                       env=env, cwd=os.path.dirname(HERE), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert " passed" in r.stdout


def test_wave_driver_for_wal_subprocess(gpu):
    """And the standalone wave kernel (MCK_CRC_ROWS=0) on the WAL records and
    the WAL writer."""
    if os.environ.get("MCK_CRC_ROWS") or os.environ.get("MCK_CRC_AUTO"):
        pytest.skip("already running a forced driver")
    env = dict(os.environ, MCK_CRC_ROWS="0")
    tests = [os.path.join(HERE, "test_wal_writer.py"),
             os.path.join(HERE, "test_crc_rows.py") + "::test_wal_record_crc_small_ragged_many"]
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-m", "gpu", "-p", "no:cacheprovider",
                        "-k", "not subprocess"] + tests,
                       env=env, cwd=os.path.dirname(HERE), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]


@pytest.mark.parametrize("lanes", ["4", "8"])
def test_row_widths_subprocess(gpu, lanes):
    """The standalone row kernel's 4- and 8-lane variants (MCK_CRC_ROW_LANES)
    on the small-span test and the generic ops."""
    if os.environ.get("MCK_CRC_ROW_LANES") or os.environ.get("MCK_CRC_AUTO"):
        pytest.skip("already running a forced width")
    env = dict(os.environ, MCK_CRC_ROWS="1", MCK_CRC_ROW_LANES=lanes)
    tests = [os.path.join(HERE, "test_crc_rows.py") + "::test_wal_record_crc_small_ragged_many"]
    tests += [os.path.join(HERE, "test_gpu_parity.py") + "::" + t for t in (
        "test_crc32c_batch_ragged", "test_sst_trailer_and_verify", "test_empty_and_zero_inputs",
        "test_large_ragged_batches_static_and_dynamic_feeds", "test_wal_record_crc_batch")]
    tests += [os.path.join(HERE, "test_blob_file.py"), os.path.join(HERE, "test_wal_writer.py")]
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-m", "gpu", "-p", "no:cacheprovider",
                        "-k", "not subprocess"] + tests,
                       env=env, cwd=os.path.dirname(HERE), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]


@pytest.mark.parametrize("mode", ["wave", "rows16", "rows8", "interleaved"])
def test_auto_kernel_forced_drivers_subprocess(gpu, mode):
    """k_crc_auto with each driver forced (its per-workgroup choice is by
    mean length, so a parity test of mixed lengths may exercise only one),
    and with the interleaved span order instead of contiguous ranges."""
    if os.environ.get("MCK_CRC_AUTO") or os.environ.get("MCK_CRC_ROWS") or os.environ.get("MCK_CRC_ORDER"):
        pytest.skip("already running a forced driver")
    env = dict(os.environ, MCK_CRC_ORDER="interleaved") if mode == "interleaved" else dict(os.environ, MCK_CRC_AUTO=mode)
    tests = [os.path.join(HERE, "test_crc_rows.py") + "::test_wal_record_crc_small_ragged_many"]
    tests += [os.path.join(HERE, "test_gpu_parity.py") + "::" + t for t in (
        "test_crc32c_batch_ragged", "test_sst_trailer_and_verify", "test_empty_and_zero_inputs",
        "test_large_ragged_batches_static_and_dynamic_feeds", "test_wal_record_crc_batch",
        "test_crc32c_known_answers_on_device", "test_builtin_checksum_batch", "test_sst_verify_large_static_feed")]
    tests += [os.path.join(HERE, "test_blob_file.py"), os.path.join(HERE, "test_wal_writer.py"),
              os.path.join(HERE, "test_sst_file.py")]
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-m", "gpu", "-p", "no:cacheprovider",
                        "-k", "not subprocess"] + tests,
                       env=env, cwd=os.path.dirname(HERE), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]

"""C++-timed latency of one small VerifyBlockChecksum batch
(tests/cpp/latency_verify.hip): mck_sst_verify_batch +
hipStreamSynchronize from C++, the call a re-pointed RetrieveMultipleBlocks
would make (<= 32 blocks, table/multiget_context.h:103).  The harness checks
its own flags (all clear, then exactly one corrupted block); the timings are
recorded, not asserted (INTEGRATION.md 2.1 cites them)."""
import json
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "tests", "cpp", "latency_verify")


def test_latency_harness_built():
    assert os.path.exists(BIN), "run __graft_entry__.build()"


@pytest.mark.gpu
def test_latency_harness_runs(gpu):
    out = subprocess.run([BIN, "300"], capture_output=True, text=True, timeout=120)
    print(out.stdout)
    print(out.stderr)
    assert out.returncode == 0, out.stdout + out.stderr
    d = json.loads(out.stdout)
    assert [r["blocks"] for r in d["rows"]] == [1, 8, 32, 64, 256]
    assert all(r["ok"] for r in d["rows"])

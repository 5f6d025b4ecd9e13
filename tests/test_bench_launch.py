"""bench.py --gpus N: a plain `python bench.py --gpus N`
starts N ranks itself (torch.distributed.run as a child process, never an
exec) and refuses more GPUs than it sees instead of timing one; under
torchrun, --gpus must equal WORLD_SIZE.  The rank launcher is driven here
with a stub rank under gloo on the CPU."""
import json
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)


@pytest.mark.parametrize("n", [2, 3])
def test_launch_ranks_runs_n_ranks(tmp_path, n):
    import bench
    out = tmp_path / "seen.json"
    env = dict(os.environ, OMP_NUM_THREADS="1")
    rc = bench.launch_ranks([str(out), str(n)], n, script=os.path.join(HERE, "_launch_stub.py"), env=env)
    assert rc == 0
    seen = json.loads(out.read_text())
    assert seen["world"] == n
    # the shares partition the batch: contiguous, disjoint, complete
    ranges = seen["ranges"]
    assert ranges[0][0] == 0 and ranges[-1][1] == 10_000
    assert all(ranges[k][1] == ranges[k + 1][0] for k in range(n - 1))
    assert seen["total"] == seen["expect_total"]
    assert seen["tmax"] == float(n)


def test_more_gpus_than_visible_is_refused():
    """No GPU in this container: `bench.py --gpus 2` must fail, not time 1."""
    import torch
    have = torch.cuda.device_count()
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(max(2, have + 1)), "--steps", "1",
                        "--warmup", "0"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "GPU(s) visible" in r.stderr


def test_gpus_must_match_world_size():
    import bench
    assert bench.check_world(None, "4") == 4
    assert bench.check_world(4, "4") == 4
    assert bench.check_world(None, None) == 1
    with pytest.raises(SystemExit):
        bench.check_world(8, "1")

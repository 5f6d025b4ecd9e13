#!/bin/bash
# round 3 re-entry: GPU suite + the headline and the few-KiB / SST lines at HEAD
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r3base}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 240 --timeout-method thread tests > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
fi
B="timeout -k 10 180 python -u bench.py --steps 20 --warmup 20 --cpu-seconds 0"
$B > $O/headline.json || exit 1
$B --workload crc32c --block-bytes 4300 --blocks 1000000 > $O/u4300.json || exit 1
$B --workload ragged --span-min 4100 --span-max 4400 --span-bytes $((4<<30)) > $O/r4100.json || exit 1
$B --workload sst > $O/sst.json || exit 1
$B --workload blob > $O/blob.json || exit 1
for f in $O/*.json; do echo "$f $(python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['roofline']['frac'], d['roofline'].get('kernel_avg_ms'))")"; done

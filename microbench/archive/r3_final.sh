#!/bin/bash
# round 3 final check on the committed tree: GPU suite, smoke, the driver's
# headline command, configs[2] / configs[3] / WAL-record lines
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r3final}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 600 --timeout-method thread tests > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/headline.json 2> $O/headline.err || exit 1
B="timeout -k 10 200 python -u bench.py --cpu-seconds 0"
$B --workload sst > $O/sst.json || exit 1
$B --workload walrec > $O/walrec.json || exit 1
$B --workload xxh3 > $O/xxh3.json || exit 1
$B --workload wal > $O/wal.json || exit 1
for f in $O/*.json; do echo "$f $(python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['roofline']['frac'], d['roofline'].get('kernel_avg_ms'))")"; done

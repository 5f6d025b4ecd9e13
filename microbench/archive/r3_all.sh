#!/bin/bash
# round 3: everything pending in one box session (boxes are scarce)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r3b}
bash microbench/r3_units3.sh ${T} || exit 1
bash microbench/r3_short.sh ${T}_short || exit 1
O=gpurun_out/${T}_wal
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py -k "wal" > $O/wal_tests.log 2>&1 || { tail -20 $O/wal_tests.log; exit 1; }
tail -1 $O/wal_tests.log
timeout -k 10 300 python -u bench.py --workload wal --steps 10 --warmup 5 --cpu-seconds 0 > $O/wal.json || exit 1
cut -c1-400 $O/wal.json

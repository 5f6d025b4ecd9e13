#!/bin/bash
# round 3 end state, part 1: GPU suite + smoke + headline (driver-shaped) +
# profiles (trace, FETCH, WRITE) of the headline and configs[2]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r3end}
O=gpurun_out/$T
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 600 --timeout-method thread tests > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/headline.json 2> $O/headline.err || exit 1
cut -c1-300 $O/headline.json
WORKLOADS="crc32c sst" 
for wl in $WORKLOADS; do
  timeout -k 10 300 bash profiles/run_profile.sh $T $wl || exit 1
done

#!/bin/bash
# round 3 end state, part 2: bench lines + profiles (trace, FETCH, WRITE) of the other workloads
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r3end}
O=gpurun_out/$T
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for wl in ${WORKLOADS:-xxh3 wal walwrite blob}; do
  timeout -k 10 300 python -u bench.py --workload $wl --cpu-seconds 0 > $O/bench_$wl.json 2> $O/bench_$wl.err || exit 1
  echo "$wl $(python3 -c "import json; d=json.load(open('$O/bench_$wl.json')); print(d['value'], d['roofline']['frac'], d['roofline'].get('kernel_avg_ms'))")"
  timeout -k 10 400 bash profiles/run_profile.sh $T $wl || exit 1
done

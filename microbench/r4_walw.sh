#!/bin/bash
# round 4: one-launch WAL writer -- parity, then A/B against the tree before
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/${1:-walw}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_wal_writer.py tests/test_wal_reader.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="timeout -k 10 180 python -u bench.py --workload walwrite --cpu-seconds 0 --steps 20 --warmup 10"
for v in head new head new; do
  if [ $v = new ]; then env -u SPEEDB_AMD_LIB $B > $O/walwrite_$v.json || exit 1
  else env SPEEDB_AMD_AB=1 SPEEDB_AMD_LIB=$PWD/microbench/_variants/$v.so $B > $O/walwrite_$v.json || exit 1; fi
  echo "$v $(python3 -c "import json; d=json.load(open('$O/walwrite_$v.json')); print(d['roofline']['frac'], d['roofline']['kernel_avg_ms'], d['verified'])")"
done
bash profiles/run_profile.sh r4walw walwrite || exit 1

#!/bin/bash
# Where the WAL writer's extra write bytes come from:
# WRITE_SIZE of k_wal_write_il for fixed 1017-B records (7 + 1017 = 1024:
# every fragment starts and ends on a 128-B line, none shares a line with its
# neighbour), fixed 1018-B records (every fragment boundary inside a line) and
# the bench's 1000-1100 B mix.  Same stream size within 0.1 %.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/walw_lines
mkdir -p $O
for c in "1017 1017" "1018 1018" "1000 1100" "1081 1081"; do
  set -- $c
  t=$1_$2
  a="--workload walwrite --cpu-seconds 0 --wal-len-min $1 --wal-len-max $2"
  timeout -k 10 180 python -u bench.py $a --steps 20 --warmup 10 > $O/bench_$t.json || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_$t -o pmc --output-format csv \
    -- python3 bench.py $a --no-verify --steps 5 --warmup 2 > $O/pmcrun_$t.txt 2>&1 || exit 1
  python3 microbench/pmc_summary.py $O/pmc_$t k_wal_write_il > $O/write_$t.txt || exit 1
  echo "$t $(python3 -c "import json; d=json.load(open('$O/bench_$t.json')); print(d['roofline']['frac'], d['config'].get('stream_bytes'), d['verified'])") $(grep WRITE_SIZE $O/write_$t.txt)"
done

#!/bin/bash
# One-pass WAL writer: parity, then walwrite A/B (default lib vs variants in $VARIANTS).
set -o pipefail
OUT=gpurun_out/${1:-r2wal80}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_wal_writer.py -m gpu -x -q --timeout 400 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
B="timeout -k 10 120 python bench.py --steps 30 --warmup 20 --workload walwrite --cpu-seconds 0"
run() { tag=$1; shift; env "$@" > $OUT/$tag.json 2>> $OUT/bench.err || exit 1; python -c "import json; d=json.load(open('$OUT/$tag.json')); print('$tag', d['value'], d['roofline']['frac'], d['roofline'].get('kernel_avg_ms'), d.get('verified'))"; }
run cur $B
for v in ${VARIANTS:-}; do run $v SPEEDB_AMD_LIB=$PWD/microbench/_variants/$v.so $B --no-verify; done
run cur_again $B

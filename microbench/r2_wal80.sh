#!/bin/bash
# One-pass WAL writer with 80-byte lane chunks (default) vs 64: parity, then walwrite A/B.
set -o pipefail
OUT=gpurun_out/${1:-r2wal80}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_wal_writer.py -m gpu -x -q --timeout 400 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
B="timeout -k 10 120 python bench.py --steps 30 --warmup 20 --workload walwrite --cpu-seconds 0"
run() { tag=$1; shift; env "$@" > $OUT/$tag.json 2>> $OUT/bench.err || exit 1; python -c "import json; d=json.load(open('$OUT/$tag.json')); print('$tag', d['value'], d['roofline']['frac'], d['roofline'].get('kernel_avg_ms'), d.get('verified'))"; }
run q80 $B
run q64 MCK_WAL_CHUNK=64 $B
run q80b $B
run q64b MCK_WAL_CHUNK=64 $B

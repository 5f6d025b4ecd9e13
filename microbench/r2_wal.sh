#!/bin/bash
# One-pass WAL writer: parity (16- and 8-lane rows), then walwrite variants.
set -o pipefail
OUT=gpurun_out/${1:-r2wal}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_wal_writer.py -m gpu -x -q --timeout 400 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
MCK_WAL_ROW_LANES=8 timeout -k 10 600 python -u -m pytest tests/test_wal_writer.py -m gpu -x -q --timeout 400 --timeout-method thread -k "not subprocess" > $OUT/pytest8.log 2>&1 || { tail -40 $OUT/pytest8.log; exit 1; }
tail -1 $OUT/pytest8.log
B="timeout -k 10 120 python bench.py --steps 30 --warmup 20 --workload walwrite"
run() { tag=$1; shift; env "$@" > $OUT/$tag.json 2>> $OUT/bench.err || exit 1; python -c "import json; d=json.load(open('$OUT/$tag.json')); print('$tag', d['value'], d['roofline']['frac'], d['roofline']['kernel_avg_ms'], d['verified'])"; }
run w16 $B
run w8 MCK_WAL_ROW_LANES=8 $B
run w16_nt0 SPEEDB_AMD_LIB=$PWD/microbench/_variants/nt0.so $B
run w8_nt0 MCK_WAL_ROW_LANES=8 SPEEDB_AMD_LIB=$PWD/microbench/_variants/nt0.so $B
run w16b $B

#!/bin/bash
# Interleaved-piece WAL writer: parity first, then walwrite A/B vs the chunk layout.
set -o pipefail
OUT=gpurun_out/${1:-r2walil}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_wal_writer.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
B="timeout -k 10 120 python bench.py --steps 30 --warmup 30 --cpu-seconds 0 --workload walwrite"
for k in 1 2; do
  $B > $OUT/il$k.json 2>> $OUT/bench.err || exit 1
  MCK_WAL_LAYOUT=chunk $B > $OUT/chunk$k.json 2>> $OUT/bench.err || exit 1
  for f in il$k chunk$k; do python -c "import json; d=json.load(open('$OUT/$f.json')); print('$f', d['value'], d['roofline']['frac'], d['ms_per_step'], d.get('verified'))"; done
done

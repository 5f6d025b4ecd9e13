#!/bin/bash
# Block KV protection: long values listed for the XXPH3 row driver (default) vs hashed in the walk.
set -o pipefail
OUT=gpurun_out/${1:-r2blk2}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_block_protection.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
B="timeout -k 10 120 python bench.py --steps 20 --warmup 10 --cpu-seconds 0 --workload blockkv"
for vb in 1000 300 100; do
  $B --kv-value-bytes $vb > $OUT/two_$vb.json 2>> $OUT/bench.err || exit 1
  MCK_BLK_TWO=0 $B --kv-value-bytes $vb > $OUT/walk_$vb.json 2>> $OUT/bench.err || exit 1
  for f in two_$vb walk_$vb; do python -c "import json; d=json.load(open('$OUT/$f.json')); print('$f', d['value'], d['roofline']['frac'], d['ms_per_step'], d.get('verified'))"; done
done

#!/bin/bash
# Row driver A/B (round 2): GPU tests, then small-span and mixed workloads
# with the row driver (MCK_CRC_ROWS=1 / default for WAL ops) vs the wave
# driver (MCK_CRC_ROWS=0).  Output: gpurun_out/$1/
set -o pipefail
OUT=gpurun_out/${1:-r2rows}
mkdir -p $OUT
B="timeout -k 10 120 python bench.py"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for w in "walrec" "ragged --span-min 512 --span-max 512" "ragged --span-min 100 --span-max 1100" "ragged --span-min 4096 --span-max 4096" "walwrite" "sst"; do
  tag=$(echo $w | tr ' ' '_' | tr -d '-')
  for m in 0 1; do
    MCK_CRC_ROWS=$m $B --workload $w --steps 30 --warmup 20 > $OUT/${tag}_rows$m.json 2>> $OUT/bench.err || exit 1
    python -c "import json,sys; d=json.load(open('$OUT/${tag}_rows$m.json')); print('$tag rows=$m', d['value'], d['roofline']['frac'], d['verified'])"
  done
done

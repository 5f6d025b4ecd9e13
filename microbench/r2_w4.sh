#!/bin/bash
# Row width for short ragged CRC spans: standalone row kernels W = 4 / 8 (interleaved
# order) vs k_crc_auto (contiguous order, and interleaved).
set -o pipefail
OUT=gpurun_out/${1:-r2w4}
mkdir -p $OUT
B="timeout -k 10 120 python bench.py --steps 30 --warmup 30 --cpu-seconds 0"
run() { tag=$1; shift; env "$@" > $OUT/$tag.json 2>> $OUT/bench.err || exit 1; python -c "import json; d=json.load(open('$OUT/$tag.json')); print('$tag', d['value'], d['roofline']['frac'], d.get('verified'))"; }
for wl in "walrec" "ragged --span-min 512 --span-max 512" "ragged --span-min 100 --span-max 300"; do
  t=$(echo $wl | tr -d ' -')
  run ${t}_auto $B --workload $wl
  run ${t}_autoilv MCK_CRC_ORDER=interleaved $B --workload $wl
  run ${t}_rows8 MCK_CRC_ROWS=1 MCK_CRC_ROW_LANES=8 $B --workload $wl
  run ${t}_rows4 MCK_CRC_ROWS=1 MCK_CRC_ROW_LANES=4 $B --workload $wl
done

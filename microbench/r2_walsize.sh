#!/bin/bash
# Per-launch overhead of the one-pass WAL writer: step time vs group-commit
# size (1, 2, 6 launches of <= ncu * 1528 fragments).
set -o pipefail
OUT=gpurun_out/${1:-r2walsize}
mkdir -p $OUT
B="timeout -k 10 120 python bench.py --steps 30 --warmup 30 --cpu-seconds 0 --no-verify --workload walwrite"
for n in 360000 720000 1440000 2097152; do
  $B --wal-records $n > $OUT/n$n.json 2>> $OUT/bench.err || exit 1
  python -c "import json; d=json.load(open('$OUT/n$n.json')); print($n, d['ms_per_step'], d['roofline']['frac'], d['config'].get('fragments'))"
done

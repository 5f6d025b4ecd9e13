#!/bin/bash
# Per-launch fixed cost vs span length: ragged CRC spans at 1 and 4 GiB.
out=gpurun_out/$1
mkdir -p $out
for sz in 4096 16384 65536; do
  for gb in 1 4; do
    timeout -k 10 200 python bench.py --workload ragged --span-min $sz --span-max $sz --span-bytes $((gb << 30)) --no-verify > $out/r_${sz}_${gb}g.json 2>/dev/null || exit 1
  done
done
for f in $out/*.json; do python3 -c "
import json; d=json.load(open('$f')); print('$f', d['value'], d['roofline']['frac'], d['roofline']['kernel_avg_ms'])"; done

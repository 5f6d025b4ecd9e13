#!/bin/bash
# SST verify mix (configs[2]) at 1, 2 and 4 GiB per image, per checksum type.
out=gpurun_out/$1
mkdir -p $out
for gb in 1 2 4; do
  for t in crc32c xxh3 both; do
    timeout -k 10 200 python bench.py --workload sst --sst-types $t --sst-bytes $((gb << 30)) --no-verify > $out/sst_${t}_${gb}g.json 2>/dev/null || exit 1
  done
done
for f in $out/*.json; do python3 -c "
import json; d=json.load(open('$f')); print('$f', d['value'], d['roofline']['frac'], d['roofline']['kernel_avg_ms'])"; done

#!/bin/bash
# Block KV: long-value threshold 512 (default) vs 241 (row-cooperative for every long value)
out=gpurun_out/$1
mkdir -p $out
for vb in 300 500; do
  for v in new t241; do
    if [ $v = t241 ]; then export SPEEDB_AMD_LIB=$PWD/microbench/_variants/long241.so; else unset SPEEDB_AMD_LIB; fi
    timeout -k 10 300 python bench.py --workload blockkv --kv-value-bytes $vb --steps 20 --warmup 10 > $out/b${vb}_$v.json 2> $out/b${vb}_$v.err || exit 1
  done
done
for f in $out/*.json; do python3 -c "
import json; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['roofline']['frac'], d['verified'])"; done

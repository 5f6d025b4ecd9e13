#!/bin/bash
# Block KV: tests + bench at 1000/300/100 B values.
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_block_protection.py > $out/t.log 2>&1 || { tail -30 $out/t.log; exit 1; }
tail -1 $out/t.log
for vb in 1000 300 100; do
  timeout -k 10 300 python bench.py --workload blockkv --kv-value-bytes $vb --steps 20 --warmup 10 > $out/b${vb}.json 2> $out/b${vb}.err || exit 1
done
for f in $out/*.json; do python3 -c "
import json; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['roofline']['frac'], d['verified'])"; done

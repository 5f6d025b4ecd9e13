#!/bin/bash
# Block KV: tests, then wave-cooperative long values (default) vs per-lane.
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_block_protection.py > $out/t.log 2>&1 || { tail -30 $out/t.log; exit 1; }
tail -1 $out/t.log
for vb in 1000 300 100; do
  for v in new lane; do
    if [ $v = lane ]; then export SPEEDB_AMD_LIB=$PWD/microbench/_variants/blklane.so; else unset SPEEDB_AMD_LIB; fi
    timeout -k 10 300 python bench.py --workload blockkv --kv-value-bytes $vb --steps 20 --warmup 10 > $out/b${vb}_$v.json 2> $out/b${vb}_$v.err || exit 1
  done
done
for f in $out/*.json; do python3 -c "
import json; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['roofline']['frac'], d['verified'])"; done

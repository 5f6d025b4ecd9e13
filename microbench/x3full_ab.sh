#!/bin/bash
# A/B: XXH3 wave driver interior full-round fast path (default) vs general units.
out=gpurun_out/$1
mkdir -p $out
B=microbench/_variants/x3full0.so
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "xxh3 or sst or builtin" > $out/t.log 2>&1 || { tail -20 $out/t.log; exit 1; }
tail -1 $out/t.log
for i in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export SPEEDB_AMD_AB=1 SPEEDB_AMD_LIB=$PWD/$B; else unset SPEEDB_AMD_LIB; fi
    timeout -k 10 120 python bench.py --workload sst --sst-types xxh3 --no-verify > $out/x3_$v$i.json 2>/dev/null || exit 1
    timeout -k 10 120 python bench.py --workload sst --no-verify > $out/sst_$v$i.json 2>/dev/null || exit 1
  done
done
for f in $out/*.json; do python3 -c "
import json; d=json.load(open('$f')); print('$f', d['value'], d['roofline']['frac'])"; done

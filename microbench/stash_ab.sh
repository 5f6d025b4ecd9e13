#!/bin/bash
# A/B: rows-driver epilogue stash (default) vs one finish per span.
out=gpurun_out/$1
mkdir -p $out
B=microbench/_variants/stash0.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_wal_reader.py > $out/t.log 2>&1 || { tail -20 $out/t.log; exit 1; }
tail -1 $out/t.log
for i in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export SPEEDB_AMD_LIB=$PWD/$B; else unset SPEEDB_AMD_LIB; fi
    timeout -k 10 120 python bench.py --workload kv --no-verify > $out/kv_$v$i.json 2>/dev/null || exit 1
    timeout -k 10 120 python bench.py --workload xxh3 --no-verify --cpu-seconds 0 > $out/x3_$v$i.json 2>/dev/null || exit 1
  done
done
for f in $out/*.json; do python3 -c "
import json; d=json.load(open('$f')); print('$f', d['value'], d['roofline']['frac'])"; done

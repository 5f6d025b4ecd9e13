#!/bin/bash
# Block KV protection: GPU tests, bench lines (1000 B and 100 B values) and a
# kernel trace, into gpurun_out/$1.  Usage (gpurun): bash microbench/blk.sh blkN
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_block_protection.py > $out/t.log 2>&1 || { tail -30 $out/t.log; exit 1; }
tail -2 $out/t.log
timeout -k 10 300 python bench.py --workload blockkv --steps 20 --warmup 10 > $out/b1000.json 2> $out/b1000.err || exit 1
timeout -k 10 300 python bench.py --workload blockkv --kv-value-bytes 100 --steps 20 --warmup 10 > $out/b100.json 2> $out/b100.err || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python bench.py --workload blockkv --kv-value-bytes 100 --steps 10 --warmup 2 --no-verify > $out/prof.log 2>&1 || exit 1
cat $out/b1000.json $out/b100.json | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['verified'], d['config']['value_bytes'])"
python3 -c "
import csv
for r in csv.DictReader(open('$out/prof/run_kernel_stats.csv')): print(r['Name'][:40], r['Calls'], float(r['AverageNs'])/1e3)"

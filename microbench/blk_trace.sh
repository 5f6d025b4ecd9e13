#!/bin/bash
# Kernel trace of the blockkv step (value bytes $2).
out=gpurun_out/$1
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python bench.py --workload blockkv --kv-value-bytes ${2:-100} --steps 10 --warmup 2 --no-verify > $out/prof.log 2>&1 || exit 1
python3 -c "
import csv
for r in csv.DictReader(open('$out/prof/run_kernel_stats.csv')): print(r['Name'][:50], r['Calls'], float(r['AverageNs'])/1e3)"

#!/bin/bash
# k_wal_write_il: source-aligned pieces (default) vs output-aligned pieces (MCK_WAL_UNALIGNED=1).
set -o pipefail
OUT=gpurun_out/${1:-r2walua}
mkdir -p $OUT
B="timeout -k 10 120 python bench.py --steps 30 --warmup 30 --cpu-seconds 0 --workload walwrite"
for k in 1 2; do
  $B > $OUT/al$k.json 2>> $OUT/bench.err || exit 1
  MCK_WAL_UNALIGNED=1 $B > $OUT/ua$k.json 2>> $OUT/bench.err || exit 1
  for f in al$k ua$k; do python -c "import json; d=json.load(open('$OUT/$f.json')); print('$f', d['value'], d['roofline']['frac'], d['ms_per_step'], d.get('verified'))"; done
done

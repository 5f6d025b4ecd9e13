#!/bin/bash
# Bench line of every workload (default flags except the CPU baseline leg).
set -o pipefail
OUT=gpurun_out/${1:-r2all}
mkdir -p $OUT
for wl in crc32c xxh3 sst wal file kv walwrite blob blockkv walrec host; do
  cpu=0; [ "$wl" = crc32c ] && cpu=12
  timeout -k 10 300 python bench.py --workload $wl --cpu-seconds $cpu > $OUT/$wl.json 2> $OUT/$wl.err || { echo "$wl failed"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$wl.json')); r=d.get('roofline') or {}; print('$wl', d['value'], d['unit'], r.get('frac'), d['ms_per_step'])"
done

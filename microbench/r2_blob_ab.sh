#!/bin/bash
# Blob-file verify (1M x 4112-B CRC spans at any offset): k_crc_auto's driver choice.
set -o pipefail
OUT=gpurun_out/${1:-r2blob}
mkdir -p $OUT
B="timeout -k 10 120 python bench.py --steps 30 --warmup 30 --cpu-seconds 0 --workload blob"
for k in 1 2; do
for m in default rows16 rows8; do
  if [ $m = default ]; then $B > $OUT/$m$k.json 2>> $OUT/bench.err || exit 1
  else MCK_CRC_AUTO=$m $B > $OUT/$m$k.json 2>> $OUT/bench.err || exit 1; fi
  python -c "import json; d=json.load(open('$OUT/$m$k.json')); print('$m$k', d['value'], d['roofline']['frac'], d['ms_per_step'])"
done
done

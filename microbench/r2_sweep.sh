#!/bin/bash
# SST per-kernel split and WAL-writer piece / auto-mode sweep.
set -o pipefail
OUT=gpurun_out/${1:-r2s}
mkdir -p $OUT
B="timeout -k 10 120 python bench.py --steps 30 --warmup 20"
run() { tag=$1; shift; env "$@" > $OUT/$tag.json 2>> $OUT/bench.err || exit 1; python -c "import json; d=json.load(open('$OUT/$tag.json')); print('$tag', d['value'], d['roofline']['frac'], d['roofline']['kernel_avg_ms'], d['verified'])"; }
run sst_crc   $B --workload sst --sst-types crc32c
run sst_xxh3  $B --workload sst --sst-types xxh3
run sst_crc_wave MCK_CRC_AUTO=wave $B --workload sst --sst-types crc32c
run sst_crc_rows16 MCK_CRC_AUTO=rows16 $B --workload sst --sst-types crc32c
run sst_xxh3_rows MCK_XXH3_DRIVER=rows $B --workload sst --sst-types xxh3
for p in 1 2 4 8 16; do run walwrite_p$p MCK_WAL_PIECES=$p $B --workload walwrite; done
run walwrite_rows8 MCK_CRC_AUTO=rows8 $B --workload walwrite

#!/bin/bash
# Where the one-pass writer's time goes: variants with parts of the output
# dropped (MCK_WAL_EXP, wrong output, timing only).
set -o pipefail
OUT=gpurun_out/${1:-r2walexp}
mkdir -p $OUT
B="timeout -k 10 120 python bench.py --steps 30 --warmup 20 --no-verify --cpu-seconds 0 --workload walwrite"
run() { tag=$1; shift; env "$@" > $OUT/$tag.json 2>> $OUT/bench.err || exit 1; python -c "import json; d=json.load(open('$OUT/$tag.json')); print('$tag', d['value'], d['roofline']['kernel_avg_ms'])"; }
run base SPEEDB_AMD_LIB=$PWD/microbench/_variants/${BASE:-base80}.so $B
for v in ${VARIANTS:-1 8 16 6}; do run exp$v SPEEDB_AMD_LIB=$PWD/microbench/_variants/exp$v.so $B; done
run base_again SPEEDB_AMD_LIB=$PWD/microbench/_variants/${BASE:-base80}.so $B

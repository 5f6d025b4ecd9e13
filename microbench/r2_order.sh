#!/bin/bash
# A/B of the k_crc_auto span order (interleaved vs MCK_CRC_ORDER=blocked)
# over ragged CRC workloads.
set -o pipefail
OUT=gpurun_out/${1:-r2order}
mkdir -p $OUT
B="timeout -k 10 120 python bench.py --steps 30 --warmup 30 --cpu-seconds 0"
run() { tag=$1; shift; env "$@" > $OUT/$tag.json 2>> $OUT/bench.err || exit 1; python -c "import json; d=json.load(open('$OUT/$tag.json')); print('$tag', d['value'], d['roofline']['frac'])"; }
for k in 1 2; do
for o in interleaved blocked; do
run walrec_$o$k MCK_CRC_ORDER=$o $B --workload walrec
run r512_$o$k MCK_CRC_ORDER=$o $B --workload ragged --span-min 512 --span-max 512
run r4k_$o$k MCK_CRC_ORDER=$o $B --workload ragged --span-min 4096 --span-max 4096
run sstcrc_$o$k MCK_CRC_ORDER=$o $B --workload sst --sst-types crc32c
done
done

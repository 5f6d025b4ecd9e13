#!/bin/bash
# k_crc_auto's "ragged 4 KiB" rule (spans of a few KiB whose last wave round is mostly
# empty -> 16-lane rows): new default vs the wave driver forced.
set -o pipefail
OUT=gpurun_out/${1:-r2auto4k}
mkdir -p $OUT
B="timeout -k 10 120 python bench.py --steps 30 --warmup 30 --cpu-seconds 0"
run() { tag=$1; shift; env "$@" > $OUT/$tag.json 2>> $OUT/bench.err || exit 1; python -c "import json; d=json.load(open('$OUT/$tag.json')); print('$tag', d['value'], d['roofline']['frac'], d.get('verified'))"; }
for k in 1 2; do
for m in auto wave; do
  E=""; [ $m = wave ] && E="MCK_CRC_AUTO=wave"
  run blob_$m$k $E $B --workload blob
  run r4100_$m$k $E $B --workload ragged --span-min 4100 --span-max 4400
  run r4k_$m$k $E $B --workload ragged --span-min 4096 --span-max 4096
  run r6k_$m$k $E $B --workload ragged --span-min 5000 --span-max 7000
  run sstcrc_$m$k $E $B --workload sst --sst-types crc32c
done
done

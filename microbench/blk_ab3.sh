#!/bin/bash
# Block KV: tests, then bench (value bytes 100 / 200 / 1000) for the default
# lib and the variants in $VARIANTS (microbench/_variants/<v>.so).
set -o pipefail
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_block_protection.py > $out/t.log 2>&1 || { tail -30 $out/t.log; exit 1; }
tail -1 $out/t.log
run() { tag=$1; vb=$2; shift 2; env "$@" timeout -k 10 300 python bench.py --workload blockkv --kv-value-bytes $vb --steps 20 --warmup 10 > $out/$tag.json 2> $out/$tag.err || exit 1; python3 -c "
import json; d=json.load(open('$out/$tag.json')); print('$tag', d['value'], d['ms_per_step'], d['roofline']['frac'], d['verified'])"; }
for vb in ${SIZES:-100 200 1000}; do
  run cur_$vb $vb
  for v in ${VARIANTS:-}; do run ${v}_$vb $vb SPEEDB_AMD_LIB=$PWD/microbench/_variants/$v.so; done
done

#!/bin/bash
# Auto kernel (per-workgroup driver choice) vs the standalone wave kernel
# (MCK_CRC_ROWS=0) on the ragged workloads.
set -o pipefail
OUT=gpurun_out/${1:-r2a}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 500 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for w in "walrec" "ragged --span-min 512 --span-max 512" "ragged --span-min 100 --span-max 1100" "ragged --span-min 1024 --span-max 1024" "ragged --span-min 2048 --span-max 2048" "ragged --span-min 4096 --span-max 4096" "ragged --span-min 16384 --span-max 16384" "walwrite" "sst" "blob"; do
  tag=$(echo $w | tr ' ' '_' | tr -d '-')
  for m in auto 0; do
    if [ $m = auto ]; then E=""; else E="MCK_CRC_ROWS=0"; fi
    env $E timeout -k 10 120 python bench.py --workload $w --steps 30 --warmup 20 > $OUT/${tag}_$m.json 2>> $OUT/bench.err || exit 1
    python -c "import json,sys; d=json.load(open('$OUT/${tag}_$m.json')); print('$tag $m', d['value'], d['roofline']['frac'], d['verified'])"
  done
done

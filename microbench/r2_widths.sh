#!/bin/bash
# Row-width A/B (MCK_CRC_ROW_LANES 4/8/16) on the small-span workloads.
set -o pipefail
OUT=gpurun_out/${1:-r2w}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_crc_rows.py tests/test_wal_writer.py -m gpu -x -q --timeout 400 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for W in 4 8 16; do
for w in "walrec" "ragged --span-min 512 --span-max 512" "ragged --span-min 100 --span-max 1100" "walwrite" "ragged --span-min 4096 --span-max 4096" ${EXTRA}; do
  tag=$(echo $w | tr ' ' '_' | tr -d '-')
  MCK_CRC_ROW_LANES=$W MCK_CRC_ROWS=1 timeout -k 10 120 python bench.py --workload $w --steps 30 --warmup 20 > $OUT/${tag}_W$W.json 2>> $OUT/bench.err || exit 1
  python -c "import json,sys; d=json.load(open('$OUT/${tag}_W$W.json')); print('W=$W $tag', d['value'], d['roofline']['frac'], d['verified'])"
done; done

#!/bin/bash
# Quick row-driver check: the row/WAL parity tests, then the small-span
# workloads on the default drivers.  Output: gpurun_out/$1/
set -o pipefail
OUT=gpurun_out/${1:-r2q}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_crc_rows.py tests/test_wal_writer.py tests/test_wal_reader.py tests/test_blob_file.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for w in "walrec" "ragged --span-min 512 --span-max 512" "ragged --span-min 100 --span-max 1100" "walwrite" ${EXTRA}; do
  tag=$(echo $w | tr ' ' '_' | tr -d '-')
  MCK_CRC_ROWS=1 timeout -k 10 120 python bench.py --workload $w --steps 30 --warmup 20 > $OUT/${tag}.json 2>> $OUT/bench.err || exit 1
  python -c "import json,sys; d=json.load(open('$OUT/${tag}.json')); print('$tag', d['value'], d['roofline']['frac'], d['verified'])"
done

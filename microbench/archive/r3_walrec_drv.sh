#!/bin/bash
# round 3: driver sweep for WAL record CRCs (100-1100 B) and 100-300-B spans
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r3wd}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
B="timeout -k 10 180 python -u bench.py --cpu-seconds 0 --steps 20 --warmup 20"
for d in auto rows4 rows8 rows16 rows1; do
  $B --crc-driver $d --workload walrec > $O/walrec_$d.json || exit 1
  $B --crc-driver $d --workload ragged --span-min 100 --span-max 300 > $O/r100_$d.json || exit 1
done
for f in $O/*.json; do echo "$f $(python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['roofline']['frac'], d['roofline'].get('kernel_avg_ms'))")"; done

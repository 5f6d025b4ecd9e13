#!/bin/bash
# round 4: row-driver width sweep on short ragged spans (this library).
#   $1 = output tag; ROWS_WL = workloads
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4rows}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
declare -A ARGS=(
  [r100]="--workload ragged --span-min 100 --span-max 300"
  [r300]="--workload ragged --span-min 300 --span-max 700"
  [walrec]="--workload walrec"
  [r512]="--workload ragged --span-min 512 --span-max 512"
  [r2k]="--workload ragged --span-min 1500 --span-max 2500"
)
B="timeout -k 10 180 python -u bench.py --cpu-seconds 0 --steps 20 --warmup 20"
for wl in ${ROWS_WL:-r100 r300 walrec r512 r2k}; do
  for d in ${ROWS_DRV:-auto rows16 rows8 rows4 rows1}; do
    $B ${ARGS[$wl]} --crc-driver $d > $O/${wl}_$d.json || exit 1
  done
done
for f in $O/*.json; do echo "$f $(python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['roofline']['frac'], d['roofline'].get('kernel_avg_ms'), d.get('verified'))")"; done

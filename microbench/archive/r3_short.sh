#!/bin/bash
# round 3: short spans (rows4 vs rows8 vs rows16), small-batch latency, SST
# per-file points (one SST file per batch: 64 / 256 MiB / 1 GiB per image)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r3short}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_crc_rows.py > $O/rows_tests.log 2>&1 || { tail -30 $O/rows_tests.log; exit 1; }
tail -1 $O/rows_tests.log
B="timeout -k 10 180 python -u bench.py --steps 20 --warmup 20 --cpu-seconds 0"
for d in rows4 rows8 rows16; do
  $B --crc-driver $d --workload ragged --span-min 100 --span-max 300 > $O/r100_$d.json || exit 1
  $B --crc-driver $d --workload walrec > $O/walrec_$d.json || exit 1
done
$B --workload ragged --span-min 100 --span-max 300 > $O/r100_auto.json || exit 1
$B --workload walrec > $O/walrec_auto.json || exit 1
$B --workload walwrite > $O/walwrite.json || exit 1
for s in 64 256 1024; do
  $B --workload sst --sst-bytes $((s<<20)) > $O/sst_${s}m.json || exit 1
done
for f in $O/*.json; do echo "$f $(python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['roofline']['frac'], d['roofline'].get('kernel_avg_ms'), d.get('verified'))")"; done
timeout -k 10 300 python -u bench.py --workload latency > $O/latency.json 2> $O/latency.err || { tail -5 $O/latency.err; exit 1; }
cat $O/latency.json

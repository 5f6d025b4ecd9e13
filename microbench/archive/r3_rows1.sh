#!/bin/bash
# round 3: one lane per span (rows1) on short ragged spans; parity first
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r3r1}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 800 --timeout-method thread "tests/test_crc_rows.py::test_auto_kernel_forced_drivers_subprocess[rows1]" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="timeout -k 10 240 python -u bench.py --cpu-seconds 0"
for d in rows1 rows4 auto; do
  $B --crc-driver $d --workload ragged --span-min 100 --span-max 300 > $O/r100_$d.json || exit 1
  $B --crc-driver $d --workload walrec > $O/walrec_$d.json || exit 1
  $B --crc-driver $d --workload ragged --span-min 1000 --span-max 3000 > $O/r1000_$d.json || exit 1
done
$B --crc-driver rows1 --workload ragged --span-min 20 --span-max 100 > $O/r20_rows1.json || exit 1
$B --workload ragged --span-min 20 --span-max 100 > $O/r20_auto.json || exit 1
for f in $O/*.json; do echo "$f $(python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['roofline']['frac'], d['roofline'].get('kernel_avg_ms'))")"; done

#!/bin/bash
# round 3: walrec / short-span lines, HEAD library vs working tree (A/B, alternating)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r3wab}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
B="timeout -k 10 180 python -u bench.py --cpu-seconds 0 --steps 20 --warmup 20"
H="env SPEEDB_AMD_LIB=$PWD/microbench/_variants/head.so"
for k in 1 2; do
  $H $B --workload walrec > $O/walrec_head$k.json || exit 1
  $B --workload walrec > $O/walrec_new$k.json || exit 1
done
$H $B --workload ragged --span-min 100 --span-max 300 > $O/r100_head.json || exit 1
$B --workload ragged --span-min 100 --span-max 300 > $O/r100_new.json || exit 1
$H $B --workload walwrite > $O/walwrite_head.json || exit 1
$B --workload walwrite > $O/walwrite_new.json || exit 1
for f in $O/*.json; do echo "$f $(python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['roofline']['frac'], d['roofline'].get('kernel_avg_ms'), d['roofline'].get('kernel'))")"; done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_sst_file.py tests/test_crc_units.py tests/test_crc_rows.py -k "not subprocess" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
$H $B --workload sst > $O/sst_head.json || exit 1
$B --workload sst > $O/sst_new.json || exit 1
$H $B --workload sst --sst-types xxh3 > $O/sstx_head.json || exit 1
$B --workload sst --sst-types xxh3 > $O/sstx_new.json || exit 1
for f in $O/sst*.json; do echo "$f $(python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['roofline']['frac'], d['roofline'].get('kernel_avg_ms'))")"; done

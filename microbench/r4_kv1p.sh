#!/bin/bash
# round 4: one-pass block KV -- parity, then one-pass vs two-pass bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/${1:-kv1p}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_block_protection.py > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
B="timeout -k 10 180 python -u bench.py --workload blockkv --cpu-seconds 0 --steps 20 --warmup 10"
for vb in 100 1000; do
  $B --kv-value-bytes $vb > $O/kv${vb}_1p.json || exit 1
  $B --kv-value-bytes $vb --kv-two-pass > $O/kv${vb}_2p.json || exit 1
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/trace100 -o t --output-format csv -- python3 bench.py --workload blockkv --kv-value-bytes 100 --cpu-seconds 0 --no-verify --steps 5 --warmup 3 > $O/trace100.txt 2>&1 || exit 1
for f in $O/*.json; do echo "$f $(python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['roofline']['frac'], d['roofline'].get('kernel_avg_ms'), d.get('verified'))")"; done
python3 - $O/trace100 <<'PY'
import csv,glob,sys
for f in glob.glob(sys.argv[1]+'/**/*kernel_stats.csv',recursive=True):
    for r in csv.DictReader(open(f)):
        print(r['Name'].split('(')[0][-40:], r['Calls'], round(float(r['AverageNs'])/1000,1))
PY

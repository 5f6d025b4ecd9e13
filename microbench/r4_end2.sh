#!/bin/bash
# Round-4 second evidence pass (after the XXH3 role split and the one-pass
# block KV entry points): parity of the touched paths, default-flag bench
# lines of the changed workloads, the small-batch latency line, and kernel
# traces + traffic of the new block KV step.
#   $1 = part (1: tests + bench lines, 2: block KV profile)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r4end2
mkdir -p $O
B="timeout -k 10 240 python -u bench.py"
case "${1:-1}" in
1)
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_block_protection.py tests/test_sst_file.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
  $B --workload sst --cpu-seconds 0 > $O/sst.json || exit 1
  $B --workload xxh3 --cpu-seconds 0 > $O/xxh3.json || exit 1
  $B --workload blockkv --cpu-seconds 0 > $O/blockkv.json || exit 1
  $B --workload blockkv --kv-value-bytes 100 --cpu-seconds 0 > $O/blockkv100.json || exit 1
  $B --workload latency > $O/latency.json || exit 1
  for f in $O/*.json; do echo "$f $(python3 -c "import json,sys; d=json.load(open('$f')); r=d.get('roofline') or {}; print(d['value'], d.get('unit'), r.get('frac'), r.get('kernel_avg_ms'), d.get('verified'))")"; done
  ;;
2)
  bash profiles/run_profile.sh r4end2 blockkv || exit 1
  bash profiles/run_profile.sh r4end2_100 blockkv --kv-value-bytes 100 || exit 1
  bash profiles/run_profile.sh r4end2 sst || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/lat_trace -o t --output-format csv -- python3 bench.py --workload latency > $O/lat_trace.txt 2>&1 || exit 1
  ;;
esac
echo "part ${1:-1} done"

#!/bin/bash
# Session C re-entry check: GPU suite, smoke, headline + kv lines
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r6c_check
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -5 $O/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
B="timeout -k 10 240 python -u bench.py"
$B > $O/crc32c.json || exit 1
$B --workload kv --cpu-seconds 0 > $O/kv.json || exit 1
$B --workload kv --kv-value-bytes 100 --cpu-seconds 0 > $O/kv100.json || exit 1
$B --workload blockkv --kv-value-bytes 100 --cpu-seconds 0 > $O/blockkv100.json || exit 1
echo "check done rc_tests=$rc"

#!/bin/bash
# Round-6 re-entry check: the restored tree's GPU tests, smoke, the default
# bench line and the WAL recovery shapes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r6_check
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
B="timeout -k 10 240 python -u bench.py"
$B > $O/default.json || exit 1
$B --workload walrecover --walrec-shape full32k --cpu-seconds 0 > $O/walrec_full32k.json || exit 1
$B --workload walrecover --walrec-shape mix --cpu-seconds 0 > $O/walrec_mix.json || exit 1
echo "check done"

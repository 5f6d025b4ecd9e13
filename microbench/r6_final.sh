#!/bin/bash
# Round-6 end state, part A: the whole GPU suite, smoke, and every bench
# line (default flags unless named) -> gpurun_out/bench_$TAG/
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
tag=${TAG:-r6final}
O=gpurun_out/bench_$tag
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
B="timeout -k 10 240 python -u bench.py"
$B > $O/crc32c.json || exit 1
for wl in xxh3 sst wal kv file walwrite blob blockkv walrec; do $B --workload $wl --cpu-seconds 0 > $O/$wl.json || exit 1; done
$B --workload blockkv --kv-value-bytes 100 --cpu-seconds 0 > $O/blockkv100.json || exit 1
$B --workload kv --kv-value-bytes 100 --cpu-seconds 0 > $O/kv100.json || exit 1
$B --workload ragged --span-min 100 --span-max 300 --cpu-seconds 0 > $O/r100.json || exit 1
$B --workload ragged --span-min 4100 --span-max 4400 --cpu-seconds 0 > $O/r4100.json || exit 1
$B --workload crc32c --blocks 1000000 --block-bytes 4300 --cpu-seconds 0 > $O/u4300.json || exit 1
$B --workload walrecover --walrec-shape full32k --cpu-seconds 0 > $O/walrecover_full32k.json || exit 1
$B --workload walrecover --walrec-shape mix --cpu-seconds 0 > $O/walrecover_mix.json || exit 1
$B --workload ragged --ragged-hash xxh3 --span-min 100 --span-max 300 --cpu-seconds 0 > $O/x3_r100.json || exit 1
$B --workload ragged --ragged-hash xxh3 --span-min 500 --span-max 1500 --cpu-seconds 0 > $O/x3_r500.json || exit 1
$B --workload xxh3 --block-bytes 100 --blocks 8388608 --cpu-seconds 0 > $O/x3_u100.json || exit 1
$B --workload host > $O/host.json || exit 1
echo "final A done"

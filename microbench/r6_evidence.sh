#!/bin/bash
# Round-6 evidence on the current tree: the whole GPU suite, smoke, the
# default bench line, configs[4] copy-inclusive (host) with its device-only
# and H2D-only legs, then kernel traces + FETCH/WRITE passes of the headline,
# WAL recovery (both shapes) and XXH3 100-300 B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
tag=${TAG:-r6ev}
O=gpurun_out/bench_$tag
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
B="timeout -k 10 300 python -u bench.py"
$B > $O/crc32c.json || exit 1
$B --workload host > $O/host.json || exit 1
$B --workload crc32c --blocks 1000000 --block-bytes 4300 --cpu-seconds 0 > $O/u4300.json || exit 1
$B --workload walrecover --walrec-shape full32k --cpu-seconds 0 > $O/walrec_full32k.json || exit 1
$B --workload walrecover --walrec-shape mix --cpu-seconds 0 > $O/walrec_mix.json || exit 1
$B --workload ragged --ragged-hash xxh3 --span-min 100 --span-max 300 --cpu-seconds 0 > $O/x3_100_300.json || exit 1
bash profiles/run_profile.sh $tag crc32c || exit 1
TRAFFIC_NAME=walrecover_full32k bash profiles/run_profile.sh ${tag}_full32k walrecover --walrec-shape full32k || exit 1
TRAFFIC_NAME=walrecover_mix bash profiles/run_profile.sh ${tag}_mix walrecover --walrec-shape mix || exit 1
TRAFFIC_NAME=r100_ragged_xxh3 bash profiles/run_profile.sh ${tag}_x3r100 ragged --ragged-hash xxh3 --span-min 100 --span-max 300 || exit 1
echo "evidence done"

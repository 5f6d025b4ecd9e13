#!/bin/bash
# round 3: the pipelined WAL record stream (configs[3]); parity first, then
# the wal bench (+ --sst-streams 1 vs 2 on the SST mix), then the traffic pass
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r3w}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_wal_reader.py tests/test_wal_writer.py tests/test_crc_rows.py -k "wal" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="timeout -k 10 240 python -u bench.py --cpu-seconds 0"
$B --workload wal > $O/wal.json || exit 1
$B --workload walwrite > $O/walwrite.json || exit 1
$B --workload sst --sst-streams 1 > $O/sst1.json || exit 1
$B --workload sst --sst-streams 2 > $O/sst2.json || exit 1
for f in $O/*.json; do echo "$f $(python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['roofline']['frac'], d['roofline'].get('kernel_avg_ms'))")"; done
bash profiles/run_profile.sh r3w wal --steps 3 --warmup 2 > $O/prof_wal.log 2>&1 || { tail -5 $O/prof_wal.log; exit 1; }
grep -h traffic_over_alg gpurun_out/prof_r3w_wal/traffic.json

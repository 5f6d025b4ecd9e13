#!/bin/bash
# round 3: the per-launch fixed cost (tiny SST images), XXH3 rows traffic
# after the last-stripe change, WAL traffic (configs[3]); parity first
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r3g}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_crc_units.py tests/test_gpu_parity.py tests/test_block_protection.py -k "units or sst or large_ragged or crc32c or xxh3 or xxph3 or kv or block" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="timeout -k 10 180 python -u bench.py --steps 20 --warmup 20 --cpu-seconds 0"
for s in 1 4 16 64 1024; do
  $B --workload sst --sst-types xxh3 --sst-bytes $((s<<20)) > $O/sstx_${s}m.json || exit 1
  $B --workload sst --sst-types crc32c --sst-bytes $((s<<20)) > $O/sstc_${s}m.json || exit 1
done
$B --workload xxh3 > $O/xxh3.json || exit 1
$B --workload kv > $O/kv.json || exit 1
for f in $O/*.json; do echo "$f $(python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['roofline']['frac'], d['roofline'].get('kernel_avg_ms'))")"; done
bash profiles/run_profile.sh r3g xxh3 > $O/prof_xxh3.log 2>&1 || { tail -5 $O/prof_xxh3.log; exit 1; }
grep -h traffic_over_alg gpurun_out/prof_r3g_xxh3/traffic.json
bash profiles/run_profile.sh r3g wal --steps 3 --warmup 2 > $O/prof_wal.log 2>&1 || { tail -5 $O/prof_wal.log; exit 1; }
grep -h traffic_over_alg gpurun_out/prof_r3g_wal/traffic.json

#!/bin/bash
# round 3: byte-balanced shares (batched length scan) vs shares by count,
# the auto driver choice, SST per-file points; parity first
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r3e}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_crc_units.py tests/test_gpu_parity.py tests/test_crc_rows.py -k "units or sst or large_ragged or crc32c or xxh3 or rows or wal" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="timeout -k 10 180 python -u bench.py --steps 20 --warmup 20 --cpu-seconds 0"
NB="env SPEEDB_AMD_LIB=$PWD/microbench/_variants/nobal.so"
$B --workload crc32c --block-bytes 4300 --blocks 1000000 > $O/u4300.json || exit 1
$B --workload ragged --span-min 4100 --span-max 4400 --span-bytes $((4<<30)) > $O/r4100.json || exit 1
$B --workload ragged --span-min 4096 --span-max 4096 --span-bytes $((4<<30)) > $O/r4096.json || exit 1
for v in bal nobal; do
  P=""; [ $v = nobal ] && P="$NB"
  $P $B --workload sst > $O/sst_$v.json || exit 1
  $P $B --workload sst --sst-types crc32c > $O/sstc_$v.json || exit 1
  $P $B --workload sst --sst-types xxh3 > $O/sstx_$v.json || exit 1
done
for s in 64 256; do $B --workload sst --sst-bytes $((s<<20)) > $O/sst_${s}m.json || exit 1; done
for f in $O/*.json; do echo "$f $(python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['roofline']['frac'], d['roofline'].get('kernel_avg_ms'))")"; done
bash profiles/run_profile.sh r3e sst > $O/prof_sst.log 2>&1 || { tail -5 $O/prof_sst.log; exit 1; }
bash profiles/run_profile.sh r3e xxh3 > $O/prof_xxh3.log 2>&1 || { tail -5 $O/prof_xxh3.log; exit 1; }
cat gpurun_out/prof_r3e_sst/traffic.json gpurun_out/prof_r3e_xxh3/traffic.json | grep -E "traffic_over_alg|kernel"

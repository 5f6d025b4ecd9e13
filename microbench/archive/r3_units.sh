#!/bin/bash
# round 3: unit-stream CRC driver -- parity, then A/B against the 4 KiB-round
# wave driver on the SST block shapes (uniform 4300, ragged 4100-4400, mix)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r3u
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_crc_units.py -k "not subprocess" > gpurun_out/r3u/units_tests.log 2>&1 || { tail -30 gpurun_out/r3u/units_tests.log; exit 1; }
tail -3 gpurun_out/r3u/units_tests.log
B="timeout -k 10 180 python -u bench.py --steps 20 --warmup 20 --cpu-seconds 0"
for mode in units wave; do
  MCK_CRC_AUTO=$mode $B --workload crc32c --block-bytes 4300 --blocks 1000000 > gpurun_out/r3u/u4300_$mode.json || exit 1
  MCK_CRC_AUTO=$mode $B --workload ragged --span-min 4100 --span-max 4400 --span-bytes $((4<<30)) > gpurun_out/r3u/r4100_$mode.json || exit 1
done
$B --workload sst --sst-types crc32c --sst-bytes $((1<<30)) > gpurun_out/r3u/sst1g_auto.json || exit 1
MCK_CRC_AUTO=wave $B --workload sst --sst-types crc32c --sst-bytes $((1<<30)) > gpurun_out/r3u/sst1g_wave.json || exit 1
$B --workload ragged --span-min 4096 --span-max 4096 --span-bytes $((4<<30)) > gpurun_out/r3u/r4096_auto.json || exit 1
$B --workload ragged --span-min 16384 --span-max 65536 --span-bytes $((4<<30)) > gpurun_out/r3u/r16_64k_auto.json || exit 1
$B > gpurun_out/r3u/headline.json || exit 1
for f in gpurun_out/r3u/*.json; do echo "$f $(python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['roofline']['frac'], d['verified'])")"; done

#!/bin/bash
# round 3: the wave driver's mini round folded into round 0 -- parity (wave
# forced on every generic CRC test), then the lines it moves
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r3fold}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_crc_rows.py -k "forced and wave" > $O/tests_wave.log 2>&1 || { tail -30 $O/tests_wave.log; exit 1; }
tail -1 $O/tests_wave.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_sst_file.py tests/test_crc_units.py tests/test_blob_file.py -k "not subprocess" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="timeout -k 10 180 python -u bench.py --cpu-seconds 0 --steps 20 --warmup 20"
H="env SPEEDB_AMD_LIB=$PWD/microbench/_variants/head.so"
for v in new head; do
  P=""; [ $v = head ] && P="$H"
  $P $B --crc-driver wave --workload crc32c --block-bytes 4300 --blocks 1000000 > $O/u4300_wave_$v.json || exit 1
  $P $B --crc-driver wave --workload ragged --span-min 4100 --span-max 4400 --span-bytes $((4<<30)) > $O/r4100_wave_$v.json || exit 1
  $P $B --workload sst --sst-types crc32c > $O/sstc_$v.json || exit 1
  $P $B --workload sst > $O/sst_$v.json || exit 1
  $P $B --crc-driver wave --workload blob > $O/blob_wave_$v.json || exit 1
done
$B --workload crc32c --block-bytes 4300 --blocks 1000000 > $O/u4300_auto.json || exit 1
for f in $O/*.json; do echo "$f $(python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['roofline']['frac'], d['roofline'].get('kernel_avg_ms'))")"; done

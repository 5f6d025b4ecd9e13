#!/bin/bash
# round 3: unit streams with 8 vs 4 unit slots per iteration vs the wave
# driver, byte-balanced workgroup shares vs shares by count (parity first),
# SQ mix of the 8-slot loop
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r3u3}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_crc_units.py tests/test_gpu_parity.py -k "units or sst or large_ragged or crc32c or xxh3" > $O/units_tests.log 2>&1 || { tail -30 $O/units_tests.log; exit 1; }
tail -1 $O/units_tests.log
B="timeout -k 10 180 python -u bench.py --steps 20 --warmup 20 --cpu-seconds 0"
V="env SPEEDB_AMD_LIB=$PWD/microbench/_variants"
for v in nu8 nu4 wave; do
  case $v in nu8) P=""; D=units;; nu4) P="$V/nu4.so"; D=units;; wave) P=""; D=wave;; esac
  $P $B --crc-driver $D --workload crc32c --block-bytes 4300 --blocks 1000000 > $O/u4300_$v.json || exit 1
  $P $B --crc-driver $D --workload ragged --span-min 4100 --span-max 4400 --span-bytes $((4<<30)) > $O/r4100_$v.json || exit 1
  $P $B --crc-driver $D --workload ragged --span-min 4096 --span-max 4096 --span-bytes $((4<<30)) > $O/r4096_$v.json || exit 1
  $P $B --crc-driver $D --workload sst --sst-types crc32c > $O/sstc_$v.json || exit 1
done
$V/nobal.so $B --crc-driver units --workload sst --sst-types crc32c > $O/sstc_nobal.json || exit 1
$B --workload sst --sst-types xxh3 > $O/sstx_bal.json || exit 1
$V/nobal.so $B --workload sst --sst-types xxh3 > $O/sstx_nobal.json || exit 1
$B --workload sst > $O/sst_bal.json || exit 1
$V/nobal.so $B --workload sst > $O/sst_nobal.json || exit 1
for f in $O/*.json; do echo "$f $(python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['roofline']['frac'], d['roofline'].get('kernel_avg_ms'))")"; done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --kernel-trace -d $O/pmc_nu8 -o pmc --output-format csv -- python3 bench.py --crc-driver units --workload crc32c --block-bytes 4300 --blocks 1000000 --steps 2 --warmup 1 --settle-ms 0 --no-verify --cpu-seconds 0 > $O/pmc_nu8.txt 2>&1 || { tail -5 $O/pmc_nu8.txt; exit 1; }

#!/bin/bash
# round 3: workgroups per CU (MCK_GRID_MULT variants) for the ragged CRC and
# XXH3 wave drivers -- the SST mix's per-workgroup byte imbalance; parity on
# the base build first (incl. rows1 auto for tiny spans)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r3gm}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_parity.py tests/test_sst_file.py -k "sst or large_ragged or crc32c or xxh3" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
SPEEDB_AMD_LIB=$PWD/microbench/_variants/gm4.so timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_parity.py -k "sst or large_ragged or xxh3" > $O/tests_gm4.log 2>&1 || { tail -30 $O/tests_gm4.log; exit 1; }
tail -1 $O/tests_gm4.log
B="timeout -k 10 240 python -u bench.py --cpu-seconds 0"
for v in base gm2 gm4; do
  L=""; [ $v != base ] && L="SPEEDB_AMD_LIB=$PWD/microbench/_variants/$v.so"
  env $L $B --workload sst --sst-types crc32c > $O/sstc_$v.json || exit 1
  env $L $B --workload sst --sst-types xxh3 > $O/sstx_$v.json || exit 1
  env $L $B --workload sst > $O/sst_$v.json || exit 1
  env $L $B --workload walrec > $O/walrec_$v.json || exit 1
  env $L $B --workload ragged --span-min 4100 --span-max 4400 --span-bytes $((4<<30)) > $O/r4100_$v.json || exit 1
done
$B --workload ragged --span-min 20 --span-max 100 > $O/r20_auto.json || exit 1
$B --workload ragged --span-min 50 --span-max 150 > $O/r50_auto.json || exit 1
$B --crc-driver rows8 --workload ragged --span-min 50 --span-max 150 > $O/r50_rows8.json || exit 1
for f in $O/*.json; do echo "$f $(python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['roofline']['frac'], d['roofline'].get('kernel_avg_ms'))")"; done

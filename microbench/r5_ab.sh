#!/bin/bash
# round 5 (copy of r4_ab.sh): parity of the ragged CRC paths, then a same-box A/B of chosen
# workloads against the round-3 library.
#   $1 = output tag; AB_WL = workloads (names below); AB_TESTS = test files
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4ab}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T="timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread"
$T ${AB_TESTS:-tests/test_crc_long.py tests/test_crc_rows.py tests/test_sst_file.py tests/test_blob_file.py} > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
declare -A ARGS=(
  [u4300]="--workload crc32c --block-bytes 4300 --blocks 1000000"
  [r4100]="--workload ragged --span-min 4100 --span-max 4400 --span-bytes $((4 << 30))"
  [r4096]="--workload ragged --span-min 4096 --span-max 4096 --span-bytes $((4 << 30))"
  [r16k]="--workload ragged --span-min 16384 --span-max 65536 --span-bytes $((4 << 30))"
  [sstc]="--workload sst --sst-types crc32c"
  [sstx]="--workload sst --sst-types xxh3"
  [sst]="--workload sst"
  [sst2]="--workload sst --sst-streams 2"
  [r300]="--workload ragged --span-min 300 --span-max 700"
  [blob]="--workload blob"
  [walrec]="--workload walrec"
  [r100]="--workload ragged --span-min 100 --span-max 300"
  [r512]="--workload ragged --span-min 512 --span-max 512"
  [kv100]="--workload blockkv --kv-value-bytes 100"
  [kv1000]="--workload blockkv --kv-value-bytes 1000"
  [walwrite]="--workload walwrite"
  [wal]="--workload wal"
  [r200]="--workload ragged --span-min 200 --span-max 500"
  [r150]="--workload ragged --span-min 150 --span-max 400"
  [r2k]="--workload ragged --span-min 2000 --span-max 3000"
  [r3k]="--workload ragged --span-min 2500 --span-max 3500"
  [r4k]="--workload ragged --span-min 3500 --span-max 4500"
  [x3u]="--workload xxh3"
  [x3u16k]="--workload xxh3 --block-bytes 16384 --blocks 65536"
  [x3u64k]="--workload xxh3 --block-bytes 65536 --blocks 16384"
  [x3u1k]="--workload xxh3 --block-bytes 1024 --blocks 1048576"
  [x3u1000]="--workload xxh3 --block-bytes 1000 --blocks 1048576"
  [kv]="--workload kv"
  [x3u1040]="--workload xxh3 --block-bytes 1040 --blocks 1048576"
  [x3u1032]="--workload xxh3 --block-bytes 1032 --blocks 1048576"
  [x3u1028]="--workload xxh3 --block-bytes 1028 --blocks 1048576"
  [x3u1088]="--workload xxh3 --block-bytes 1088 --blocks 1048576"
  [x3u2k]="--workload xxh3 --block-bytes 2048 --blocks 524288"
  [cu512]="--workload crc32c --block-bytes 512 --blocks 2097152"
  [cu1k]="--workload crc32c --block-bytes 1024 --blocks 1048576"
  [cu2k]="--workload crc32c --block-bytes 2048 --blocks 524288"
  [cu16k]="--workload crc32c --block-bytes 16384 --blocks 65536"
  [r512u]="--workload ragged --span-min 512 --span-max 512"
  [r1ku]="--workload ragged --span-min 1024 --span-max 1024"
  [r2ku]="--workload ragged --span-min 2048 --span-max 2048"
  [r57]="--workload ragged --span-min 500 --span-max 700"
  [r49]="--workload ragged --span-min 400 --span-max 900"
  [r113]="--workload ragged --span-min 100 --span-max 1300"
  [r48]="--workload ragged --span-min 400 --span-max 800"
  [r38]="--workload ragged --span-min 300 --span-max 800"
  [w39]="--workload walrec --span-min 300 --span-max 900"
  [r611]="--workload ragged --span-min 600 --span-max 1100"
  [crc]="--workload crc32c"
  [file]="--workload file"
)
B="timeout -k 10 180 python -u bench.py --cpu-seconds 0 --steps 20 --warmup 20"
V=$PWD/microbench/_variants
for v in ${AB_VARIANTS:-r3base new}; do
  for wl in ${AB_WL:-r4100 r16k sstc blob}; do
    if [ $v = new ]; then env -u SPEEDB_AMD_LIB $B ${ARGS[$wl]} > $O/${wl}_$v.json || exit 1
    else env SPEEDB_AMD_AB=1 SPEEDB_AMD_LIB=$V/$v.so $B ${ARGS[$wl]} > $O/${wl}_$v.json || exit 1; fi
  done
done
for f in $O/*.json; do echo "$f $(python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['roofline']['frac'], d['roofline'].get('kernel_avg_ms'), d.get('verified'))")"; done

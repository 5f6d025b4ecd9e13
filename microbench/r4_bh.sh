#!/bin/bash
# round 4: the body/head CRC driver -- parity (forced for every ragged batch)
# then same-box A/B against the round-3 library
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4bh}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_crc_rows.py -k "forced and bh" > $O/bh_tests.log 2>&1 || { tail -60 $O/bh_tests.log; exit 1; }
tail -3 $O/bh_tests.log
B="timeout -k 10 180 python -u bench.py --cpu-seconds 0 --steps 20 --warmup 20"
V=$PWD/microbench/_variants
for v in r3base bh; do
  if [ $v = r3base ]; then P="env SPEEDB_AMD_LIB=$V/r3base.so"; D=auto; else P=""; D=bh; fi
  $P $B --crc-driver $D --workload crc32c --block-bytes 4300 --blocks 1000000 > $O/u4300_$v.json || exit 1
  $P $B --crc-driver $D --workload ragged --span-min 4100 --span-max 4400 --span-bytes $((4<<30)) > $O/r4100_$v.json || exit 1
  $P $B --crc-driver $D --workload ragged --span-min 4096 --span-max 4096 --span-bytes $((4<<30)) > $O/r4096_$v.json || exit 1
  $P $B --crc-driver $D --workload sst --sst-types crc32c > $O/sstc_$v.json || exit 1
  $P $B --crc-driver $D --workload blob > $O/blob_$v.json || exit 1
  $P $B --crc-driver $D --workload ragged --span-min 16384 --span-max 65536 --span-bytes $((4<<30)) > $O/r16k_$v.json || exit 1
done
$B --workload sst --sst-types crc32c > $O/sstc_auto.json || exit 1
$B --workload crc32c --block-bytes 4300 --blocks 1000000 > $O/u4300_auto.json || exit 1
for f in $O/*.json; do echo "$f $(python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['roofline']['frac'], d['roofline'].get('kernel_avg_ms'))")"; done

#!/bin/bash
# round 4: the body/head CRC driver + the windowed row kernel -- parity
# (every ragged path, each driver forced), then same-box A/B against the
# round-3 library
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4bh}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T="timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread"
$T tests/test_crc_long.py tests/test_crc_rows.py tests/test_gpu_parity.py tests/test_sst_file.py tests/test_blob_file.py tests/test_block_protection.py > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
B="timeout -k 10 180 python -u bench.py --cpu-seconds 0 --steps 20 --warmup 20"
V=$PWD/microbench/_variants
for v in r3base new; do
  if [ $v = r3base ]; then P="env SPEEDB_AMD_AB=1 SPEEDB_AMD_LIB=$V/r3base.so"; else P=""; fi
  $P $B --workload crc32c --block-bytes 4300 --blocks 1000000 > $O/u4300_$v.json || exit 1
  $P $B --workload ragged --span-min 4100 --span-max 4400 --span-bytes $((4<<30)) > $O/r4100_$v.json || exit 1
  $P $B --workload ragged --span-min 4096 --span-max 4096 --span-bytes $((4<<30)) > $O/r4096_$v.json || exit 1
  $P $B --workload sst --sst-types crc32c > $O/sstc_$v.json || exit 1
  $P $B --workload sst --sst-types xxh3 > $O/sstx_$v.json || exit 1
  $P $B --workload sst > $O/sst_$v.json || exit 1
  $P $B --workload blob > $O/blob_$v.json || exit 1
  $P $B --workload ragged --span-min 16384 --span-max 65536 --span-bytes $((4<<30)) > $O/r16k_$v.json || exit 1
  $P $B --workload walrec > $O/walrec_$v.json || exit 1
  $P $B --workload ragged --span-min 100 --span-max 300 > $O/r100_$v.json || exit 1
  $P $B --workload ragged --span-min 512 --span-max 512 > $O/r512_$v.json || exit 1
  $P $B --workload blockkv --kv-value-bytes 100 > $O/kv100_$v.json || exit 1
  $P $B --workload blockkv --kv-value-bytes 1000 > $O/kv1000_$v.json || exit 1
done
for f in $O/*.json; do echo "$f $(python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['roofline']['frac'], d['roofline'].get('kernel_avg_ms'), d.get('verified'))")"; done

#!/bin/bash
# round 3: one k_crc_auto launch per batch (windows of the descriptor cache
# inside the workgroup) -- the generic CRC parity tests on every forced
# driver, then the short-span lines against HEAD
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r3one}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 800 --timeout-method thread tests/test_crc_rows.py tests/test_gpu_parity.py tests/test_crc_units.py tests/test_blob_file.py tests/test_sst_file.py tests/test_wal_reader.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="timeout -k 10 180 python -u bench.py --cpu-seconds 0 --steps 20 --warmup 20"
H="env SPEEDB_AMD_LIB=$PWD/microbench/_variants/head.so"
for v in new head; do
  P=""; [ $v = head ] && P="$H"
  $P $B --workload walrec > $O/walrec_$v.json || exit 1
  $P $B --workload ragged --span-min 100 --span-max 300 > $O/r100_$v.json || exit 1
  $P $B --workload ragged --span-min 512 --span-max 512 > $O/r512_$v.json || exit 1
  $P $B --workload crc32c --block-bytes 4300 --blocks 1000000 > $O/u4300_$v.json || exit 1
  $P $B --workload blob > $O/blob_$v.json || exit 1
  $P $B --workload ragged --span-min 4096 --span-max 4096 --span-bytes $((4<<30)) > $O/r4096_$v.json || exit 1
  $P $B --workload sst --sst-types crc32c > $O/sstc_$v.json || exit 1
done
for f in $O/*.json; do echo "$f $(python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['roofline']['frac'], d['roofline'].get('kernel_avg_ms'))")"; done

#!/bin/bash
# round 4: same-box baseline, round-3 library vs the wsum fix
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4base}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
B="timeout -k 10 180 python -u bench.py --cpu-seconds 0 --steps 20 --warmup 20"
V=$PWD/microbench/_variants
for v in r3base wsum; do
  P="env SPEEDB_AMD_AB=1 SPEEDB_AMD_LIB=$V/$v.so"
  $P $B --workload sst > $O/sst_$v.json || exit 1
  $P $B --workload sst --sst-types crc32c > $O/sstc_$v.json || exit 1
  $P $B --workload sst --sst-types xxh3 > $O/sstx_$v.json || exit 1
  $P $B --workload crc32c --block-bytes 4300 --blocks 1000000 > $O/u4300_$v.json || exit 1
  $P $B --workload ragged --span-min 4100 --span-max 4400 --span-bytes $((4<<30)) > $O/r4100_$v.json || exit 1
  $P $B --workload ragged --span-min 4096 --span-max 4096 --span-bytes $((4<<30)) > $O/r4096_$v.json || exit 1
  $P $B --workload walrec > $O/walrec_$v.json || exit 1
  $P $B --workload ragged --span-min 100 --span-max 300 > $O/r100_$v.json || exit 1
done
for f in $O/*.json; do echo "$f $(python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['roofline']['frac'], d['roofline'].get('kernel_avg_ms'))")"; done

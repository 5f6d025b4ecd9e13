#!/bin/bash
# round 3: byte-balanced workgroup shares (share_by_bytes) -- parity, then the SST lines
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r3bal}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_sst_file.py tests/test_crc_units.py tests/test_blob_file.py -k "not subprocess" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="timeout -k 10 180 python -u bench.py --cpu-seconds 0"
$B --workload sst > $O/sst.json || exit 1
$B --workload sst --sst-types crc32c > $O/sstc.json || exit 1
$B --workload sst --sst-types xxh3 > $O/sstx.json || exit 1
$B --workload sst --sst-bytes $((256<<20)) > $O/sst256m.json || exit 1
$B --workload crc32c --block-bytes 4300 --blocks 1000000 > $O/u4300.json || exit 1
$B --workload ragged --span-min 4100 --span-max 4400 --span-bytes $((4<<30)) > $O/r4100.json || exit 1
$B --workload walrec > $O/walrec.json || exit 1
$B --workload blob > $O/blob.json || exit 1
$B > $O/headline.json || exit 1
for f in $O/*.json; do echo "$f $(python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['roofline']['frac'], d['roofline'].get('kernel_avg_ms'))")"; done

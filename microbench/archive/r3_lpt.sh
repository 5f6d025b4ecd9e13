#!/bin/bash
# round 3: longest-first tickets for the wave driver (the SST mix's tail);
# parity first (incl. the forced wave driver), then the SST sizes and the
# wave-driver shapes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r3l}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_parity.py tests/test_sst_file.py tests/test_crc_rows.py tests/test_block_protection.py -k "sst or large_ragged or crc32c or wave or block or wal" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="timeout -k 10 240 python -u bench.py --cpu-seconds 0"
$B --workload sst > $O/sst.json || exit 1
for s in 1 64 256; do
  $B --steps 20 --warmup 20 --workload sst --sst-types crc32c --sst-bytes $((s<<20)) > $O/sstc_${s}m.json || exit 1
done
$B --workload sst --sst-types crc32c > $O/sstc_1024m.json || exit 1
$B --workload sst --sst-types xxh3 > $O/sstx_1024m.json || exit 1
$B --workload ragged --span-min 4096 --span-max 4096 --span-bytes $((4<<30)) > $O/r4096.json || exit 1
$B --workload ragged --span-min 16384 --span-max 65536 --span-bytes $((4<<30)) > $O/r16_64k.json || exit 1
$B --workload blob > $O/blob.json || exit 1
for f in $O/*.json; do echo "$f $(python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['roofline']['frac'], d['roofline'].get('kernel_avg_ms'))")"; done

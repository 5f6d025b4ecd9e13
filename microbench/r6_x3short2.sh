#!/bin/bash
# Round 6: short-span XXH3 on rows -- parity, then the short-span bench
# lines and the workloads whose kernels hold the short pass (SST mix, KV,
# WAL recovery mix).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/${TAG:-r6_x3s2}
mkdir -p $O
T="timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
$T tests/test_xxh3_short.py tests/test_crc_long.py tests/test_gpu_parity.py tests/test_wal_recover.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
B="timeout -k 10 240 python -u bench.py --cpu-seconds 0"
$B --workload ragged --ragged-hash xxh3 --span-min 100 --span-max 300 > $O/x3_100_300.json || exit 1
$B --workload ragged --ragged-hash xxh3 --span-min 16 --span-max 240 > $O/x3_16_240.json || exit 1
$B --workload ragged --ragged-hash xxh3 --span-min 241 --span-max 600 > $O/x3_241_600.json || exit 1
$B --workload walrecover --walrec-shape mix > $O/walrec_mix.json || exit 1
$B --workload sst > $O/sst.json || exit 1
$B --workload kv > $O/kv.json || exit 1
for f in $O/*.json; do python3 -c "
import json,sys
for l in open('$f'):
    if l.startswith('{'):
        d=json.loads(l); print('$f', d['value'], d['roofline']['frac'], d.get('verified'))"; done
echo done

#!/bin/bash
# Round 6: XXH3 short spans baseline (ragged 100-300 B, 16-240 B, 241-600 B)
# + the block-protection verify fallback test.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/${TAG:-r6_x3s}
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_block_protection.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
B="timeout -k 10 240 python -u bench.py --workload ragged --ragged-hash xxh3 --cpu-seconds 0"
$B --span-min 100 --span-max 300 > $O/x3_100_300.json || exit 1
$B --span-min 16 --span-max 240 > $O/x3_16_240.json || exit 1
$B --span-min 241 --span-max 600 > $O/x3_241_600.json || exit 1
timeout -k 10 240 python -u bench.py --workload ragged --span-min 100 --span-max 300 --cpu-seconds 0 > $O/crc_100_300.json || exit 1
for f in $O/*.json; do python3 -c "
import json,sys
for l in open('$f'):
    if l.startswith('{'):
        d=json.loads(l); print('$f', d['value'], d['roofline']['frac'], d.get('verified'))"; done
echo done

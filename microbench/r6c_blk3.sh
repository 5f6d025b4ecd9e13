#!/bin/bash
# Interleaved slots in the product: the GPU suite, then the block KV A/B
# against the previous layout (blkold) with FETCH/WRITE passes.
set -uo pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/${OUT:-r6c_blk3}
mkdir -p $o
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
VARS="blkold" OUT=${OUT:-r6c_blk3} bash microbench/ab_blk.sh || exit 1
TRAFFIC_NAME=100_blockkv bash profiles/run_profile.sh ${OUT:-r6c} blockkv --kv-value-bytes 100 || exit 1
bash profiles/run_profile.sh ${OUT:-r6c} blockkv || exit 1
timeout -k 10 240 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $o/smoke.log 2>&1 || exit 1
timeout -k 10 240 python3 -u bench.py > $o/crc32c.json || exit 1
echo "blk3 done"

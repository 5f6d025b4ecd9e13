#!/bin/bash
# Interleaved slots in the product: the GPU suite, then the block KV A/B
# against the previous layout (blkold) with FETCH/WRITE passes.
set -uo pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/r6c_blk3
mkdir -p $o
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
VARS="blkold" OUT=r6c_blk3 bash microbench/ab_blk.sh

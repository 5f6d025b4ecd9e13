#!/bin/bash
# Variant parity (block protection GPU tests on the variant library), then ab_blk.sh
set -uo pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/${OUT:-r6c_blk}
mkdir -p $o
for v in $VARS; do
  SPEEDB_AMD_LIB=$PWD/microbench/_variants/$v.so SPEEDB_AMD_AB=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_block_protection.py -m gpu > $o/tests_$v.log 2>&1 || { tail -30 $o/tests_$v.log; exit 1; }
  tail -1 $o/tests_$v.log
done
bash microbench/ab_blk.sh

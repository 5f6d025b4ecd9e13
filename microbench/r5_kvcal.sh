#!/bin/bash
# Block KV read-traffic calibration: FETCH_SIZE next to TCC_EA0 read request
# counts (all requests, and the 32-B ones) per kernel of the step, 100-B and
# 1000-B values (the WAL replay's calibration, DESIGN.md 5, for gathers).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/kvcal
mkdir -p $O
for vb in 100 1000; do
  A="--workload blockkv --kv-value-bytes $vb --cpu-seconds 0 --no-verify --steps 3 --warmup 2"
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/f$vb -o pmc --output-format csv -- python3 bench.py $A > $O/bf$vb.txt 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --kernel-trace -d $O/q$vb -o pmc --output-format csv -- python3 bench.py $A > $O/bq$vb.txt 2>&1 || exit 1
  echo "== $vb"; python3 microbench/pmc_summary.py $O/f$vb k_block k_blk | tee $O/f$vb.txt; python3 microbench/pmc_summary.py $O/q$vb k_block k_blk | tee $O/q$vb.txt
done

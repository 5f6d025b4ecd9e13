#!/bin/bash
# Instruction mix, wait states and addresser load of one bench workload's
# kernel: three --pmc passes (each within the per-block counter limits).
#   SQP_OUT = output dir under gpurun_out; SQP_K = kernel name substring;
#   remaining args = bench.py arguments
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${SQP_OUT:-sqprof}
mkdir -p $O
A="$* --cpu-seconds 0 --no-verify --steps 5 --warmup 3"
P="timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -o pmc"
$P --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/sq1 -- python3 bench.py $A > $O/b1.txt 2>&1 || exit 1
$P --pmc SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_WAIT_ANY -d $O/sq2 -- python3 bench.py $A > $O/b2.txt 2>&1 || exit 1
$P --pmc TA_TA_BUSY_sum TA_BUSY_max GRBM_GUI_ACTIVE -d $O/ta -- python3 bench.py $A > $O/b3.txt 2>&1 || exit 1
python3 microbench/pmc_summary.py $O ${SQP_K:-k_} > $O/summary.txt || exit 1
cat $O/summary.txt

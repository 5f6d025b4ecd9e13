#!/bin/bash
# block KV (100-B values) instruction mix and texture-addresser load
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${KV_OUT:-kvprof}
mkdir -p $O
A="--workload blockkv --kv-value-bytes ${KV_BYTES:-100} --cpu-seconds 0 --no-verify --steps 5 --warmup 3"
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --kernel-trace -d $O/sq -o pmc --output-format csv -- python3 bench.py $A > $O/b_sq.txt 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TA_BUSY_max GRBM_GUI_ACTIVE --kernel-trace -d $O/ta -o pmc --output-format csv -- python3 bench.py $A > $O/b_ta.txt 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/fetch -o pmc --output-format csv -- python3 bench.py $A > $O/b_f.txt 2>&1 || exit 1
echo done

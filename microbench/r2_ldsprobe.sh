#!/bin/bash
# LDS bank conflicts / instruction mix of the CRC drivers (one PMC pass per workload).
set -o pipefail
OUT=gpurun_out/${1:-r2lds}
mkdir -p $OUT
export TMPDIR=/tmp
for wl in ${WORKLOADS:-walrec crc32c}; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace -d $OUT/$wl -o pmc --output-format csv -- python3 bench.py --workload $wl --steps 5 --warmup 2 --cpu-seconds 0 --no-verify > $OUT/$wl.txt 2>&1 || exit 1
done
echo done

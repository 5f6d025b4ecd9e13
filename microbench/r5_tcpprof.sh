#!/bin/bash
# L1 (TCP) request counts next to SQ/TA counters for one workload, the
# in-tree library against a variant (VAR=_variants/<v>.so).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TP_OUT:-tcpprof}
mkdir -p $O
A="$* --cpu-seconds 0 --no-verify --steps 5 --warmup 3"
P="timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -o pmc"
for v in new ${VAR:-}; do
  if [ $v = new ]; then E="env -u SPEEDB_AMD_LIB"; else E="env SPEEDB_AMD_AB=1 SPEEDB_AMD_LIB=$PWD/microbench/_variants/$v.so"; fi
  $E $P --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TA_TA_BUSY_sum GRBM_GUI_ACTIVE -d $O/$v/tcp -- python3 bench.py $A > $O/$v.b1.txt 2>&1 || exit 1
  $E $P --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS -d $O/$v/sq -- python3 bench.py $A > $O/$v.b2.txt 2>&1 || exit 1
  echo "== $v"; python3 microbench/pmc_summary.py $O/$v ${TP_K:-k_crc_ragged} | tee $O/$v.summary.txt
done

#!/bin/bash
# Profile the headline bench on the GPU box (run from the repo root via gpurun).
#   $1 = tag (output goes to gpurun_out/prof_<tag>/)
# Pass 1: kernel trace + stats (per-kernel average duration).
# Pass 2/3: PMC counters, one block per pass (FETCH_SIZE costs 3 TCC slots):
#   TCC FETCH_SIZE / WRITE_SIZE for the HBM traffic, SQ counters for the
#   instruction mix.  Collected with --kernel-trace only (no sys/runtime trace).
set -euo pipefail
tag=${1:-run}
out=gpurun_out/prof_${tag}
mkdir -p "$out"
export TMPDIR=/tmp
args="--steps 10 --warmup 2 --cpu-seconds 0 --no-verify"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/trace" -o trace --output-format csv -- python3 bench.py $args > "$out/bench_trace.txt" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$out/pmc_fetch" -o pmc --output-format csv -- python3 bench.py $args > "$out/bench_fetch.txt" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$out/pmc_write" -o pmc --output-format csv -- python3 bench.py $args > "$out/bench_write.txt" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --kernel-trace -d "$out/pmc_sq" -o pmc --output-format csv -- python3 bench.py $args > "$out/bench_sq.txt" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE --kernel-trace -d "$out/pmc_sq2" -o pmc --output-format csv -- python3 bench.py $args > "$out/bench_sq2.txt" 2>&1
echo "profile done: $out"

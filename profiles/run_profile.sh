#!/bin/bash
# Profile one bench workload on the GPU box (run from the repo root via gpurun).
#   $1 = tag, $2 = workload (crc32c|xxh3|sst|wal), rest = extra bench args
# Output: gpurun_out/prof_<tag>_<workload>/
# Pass 1: kernel trace + stats (per-kernel average duration).
# Passes 2/3: TCC FETCH_SIZE and WRITE_SIZE, one per pass (they do not fit
#   together), --kernel-trace only (never with sys/runtime trace).
# Pass 4 (PROFILE_SQ=1): SQ instruction mix.
set -euo pipefail
tag=${1:-run}
wl=${2:-crc32c}
shift 2 || true
out=gpurun_out/prof_${tag}_${wl}
mkdir -p "$out"
export TMPDIR=/tmp
args="--workload $wl --cpu-seconds 0 --no-verify $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/trace" -o trace --output-format csv -- python3 bench.py $args > "$out/bench_trace.txt" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$out/pmc_fetch" -o pmc --output-format csv -- python3 bench.py $args > "$out/bench_fetch.txt" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$out/pmc_write" -o pmc --output-format csv -- python3 bench.py $args > "$out/bench_write.txt" 2>&1
if [ "${PROFILE_SQ:-0}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --kernel-trace -d "$out/pmc_sq" -o pmc --output-format csv -- python3 bench.py $args > "$out/bench_sq.txt" 2>&1
fi
tn=${TRAFFIC_NAME:-$wl}
python3 profiles/pmc_to_traffic.py "$out" "$wl" "$tn" > "$out/traffic.json"
cp profiles/traffic_${tn}.json "$out/" 2>/dev/null || true
echo "profile done: $out"

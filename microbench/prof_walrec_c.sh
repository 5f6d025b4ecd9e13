set -uo pipefail
export TMPDIR=/tmp
o=gpurun_out/r6e
mkdir -p $o
for sh in full32k mix; do
  mkdir -p $o/$sh
  A="--workload walrecover --walrec-shape $sh --steps 20 --warmup 5 --settle-ms 100 --cpu-seconds 0 --no-verify"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/$sh/trace -o trace --output-format csv -- python3 bench.py $A > $o/$sh/bench_trace.txt 2>&1 || exit 1
  timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $o/$sh/pmc_fetch -o pmc --output-format csv -- python3 bench.py $A > $o/$sh/bench_fetch.txt 2>&1 || exit 1
  timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $o/$sh/pmc_write -o pmc --output-format csv -- python3 bench.py $A > $o/$sh/bench_write.txt 2>&1 || exit 1
  timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --kernel-trace -d $o/$sh/pmc_sq -o pmc --output-format csv -- python3 bench.py $A > $o/$sh/bench_sq.txt 2>&1 || exit 1
done
echo ok

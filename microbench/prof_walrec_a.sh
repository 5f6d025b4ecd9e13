set -uo pipefail
export TMPDIR=/tmp
o=gpurun_out/r6c
mkdir -p $o
A="--workload walrecover --walrec-shape full32k --steps 10 --warmup 5 --settle-ms 100 --no-verify"
timeout -k 10 120 python3 bench.py $A > $o/t.json 2>&1 || exit 1
MCK_WALREC_CHUNK=1 timeout -k 10 120 python3 bench.py $A > $o/c.json 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $o/fetch_t -o pmc --output-format csv -- python3 bench.py $A > $o/ft.txt 2>&1 || exit 1
MCK_WALREC_CHUNK=1 timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $o/fetch_c -o pmc --output-format csv -- python3 bench.py $A > $o/fc.txt 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --kernel-trace -d $o/sq_t -o pmc --output-format csv -- python3 bench.py $A > $o/sq.txt 2>&1 || exit 1
echo ok

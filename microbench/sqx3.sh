# SQ instruction mix: XXH3 wave vs rows driver at 4 KiB spans
set -e
mkdir -p gpurun_out/sqx3
export TMPDIR=/tmp
L=speedb_amd/libspeedb_amd.so
for drv in wave rows; do
  MCK_XXH3_DRIVER=$drv timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --kernel-trace -d gpurun_out/sqx3/$drv -o pmc --output-format csv -- python3 microbench/ab.py $L --kind xxh3 --block 4096 --blocks 1048576 --rounds 2 --iters 3 > gpurun_out/sqx3/$drv.txt 2>&1
done
echo done

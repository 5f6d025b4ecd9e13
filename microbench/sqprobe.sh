# SQ instruction mix: generic (ragged) vs uniform CRC driver at 4 KiB spans
set -e
mkdir -p gpurun_out/sq
export TMPDIR=/tmp
L=speedb_amd/libspeedb_amd.so
for mode in ragged uniform; do
  fl=""; [ $mode = ragged ] && fl="--ragged"
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --kernel-trace -d gpurun_out/sq/$mode -o pmc --output-format csv -- python3 microbench/ab.py $L --kind crc32c --block 4096 --blocks 1048576 --rounds 2 --iters 3 $fl > gpurun_out/sq/$mode.txt 2>&1
done
echo done

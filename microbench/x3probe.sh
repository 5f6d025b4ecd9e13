# XXH3 driver probe: uniform 4 KiB / 64 KiB and the SST-shaped mix, rows vs wave
set -e
mkdir -p gpurun_out
L=speedb_amd/libspeedb_amd.so
o=gpurun_out/x3probe.log
: > $o
for drv in wave rows; do
  echo "== $drv 4K" >> $o; MCK_XXH3_DRIVER=$drv timeout -k 10 120 python microbench/ab.py $L --kind xxh3 >> $o 2>&1
  echo "== $drv 64K" >> $o; MCK_XXH3_DRIVER=$drv timeout -k 10 120 python microbench/ab.py $L --kind xxh3 --block 65536 --blocks 16384 >> $o 2>&1
  echo "== $drv mix" >> $o; MCK_XXH3_DRIVER=$drv timeout -k 10 120 python microbench/ab.py $L --kind xxh3 --mixed --blocks 262144 >> $o 2>&1
done
echo "== crc mix" >> $o; timeout -k 10 120 python microbench/ab.py $L --kind crc32c --mixed --blocks 262144 >> $o 2>&1
echo "== crc 64K" >> $o; timeout -k 10 120 python microbench/ab.py $L --kind crc32c --block 65536 --blocks 16384 >> $o 2>&1
cat $o

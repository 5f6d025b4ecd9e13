# ragged-mix alignment probe: XXH3 span starts at 1 / 4 / 8 / 16-byte alignment
set -e
mkdir -p gpurun_out
L=speedb_amd/libspeedb_amd.so
o=gpurun_out/alprobe.log
: > $o
for al in 1 4 8 16; do
  echo "== xxh3 mix align=$al" >> $o; timeout -k 10 120 python microbench/ab.py $L --kind xxh3 --mixed --blocks 262144 --align $al --rounds 11 >> $o 2>&1
done
echo "== xxh3 uniform 4096+4 stride" >> $o; timeout -k 10 120 python microbench/ab.py $L --kind xxh3 --block 4100 --blocks 262144 >> $o 2>&1
echo "== xxh3 uniform 4096+1 stride" >> $o; timeout -k 10 120 python microbench/ab.py $L --kind xxh3 --block 4097 --blocks 262144 >> $o 2>&1
echo "== xxh3 uniform 4096+16 stride" >> $o; timeout -k 10 120 python microbench/ab.py $L --kind xxh3 --block 4112 --blocks 262144 >> $o 2>&1
cat $o

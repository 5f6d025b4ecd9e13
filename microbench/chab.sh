# CRC lookup chains per lane: 1 vs 2 (row-T era)
set -e
o=gpurun_out/chab.log
: > $o
for v in 1 2 1 2; do
  cp microbench/mb_lib_ch$v.so speedb_amd/libspeedb_amd.so
  for w in crc32c sst wal; do
    echo "== $w chains=$v" >> $o; timeout -k 10 180 python bench.py --workload $w --cpu-seconds 0 >> $o 2>&1
  done
done
cp microbench/mb_lib_ch2.so speedb_amd/libspeedb_amd.so
cat $o

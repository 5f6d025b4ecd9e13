# generic CRC driver with row-transposed loads: parity (T build), then A/B
set -e
mkdir -p gpurun_out
o=gpurun_out/gtab.log
: > $o
cp microbench/mb_lib_gt1.so speedb_amd/libspeedb_amd.so
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gt_pytest.log 2>&1 || { tail -40 gpurun_out/gt_pytest.log; exit 1; }
tail -2 gpurun_out/gt_pytest.log >> $o
A="microbench/mb_lib_gt0.so microbench/mb_lib_gt1.so"
echo "== crc mix" >> $o; timeout -k 10 120 python microbench/ab.py $A --kind crc32c --mixed --blocks 262144 --rounds 15 >> $o 2>&1
echo "== ragged 4K" >> $o; timeout -k 10 120 python microbench/ab.py $A --kind crc32c --block 4096 --blocks 1048576 --ragged --rounds 11 >> $o 2>&1
echo "== ragged 64K" >> $o; timeout -k 10 120 python microbench/ab.py $A --kind crc32c --block 65536 --blocks 65536 --ragged --rounds 11 >> $o 2>&1
for v in 1 0; do
  cp microbench/mb_lib_gt$v.so speedb_amd/libspeedb_amd.so
  for w in sst blob walwrite; do
    echo "== $w gt=$v" >> $o; timeout -k 10 180 python bench.py --workload $w --cpu-seconds 0 >> $o 2>&1
  done
done
cp microbench/mb_lib_gt0.so speedb_amd/libspeedb_amd.so
cat $o

# span setup one span ahead (crc_drive AHEAD): parity, then A/B
set -e
mkdir -p gpurun_out
o=gpurun_out/ahab.log
: > $o
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ah_pytest.log 2>&1 || { tail -40 gpurun_out/ah_pytest.log; exit 1; }
tail -2 gpurun_out/ah_pytest.log >> $o
A="microbench/mb_lib_ah0.so microbench/mb_lib_ah1.so"
echo "== ragged 4K (static feed)" >> $o; timeout -k 10 120 python microbench/ab.py $A --kind crc32c --block 4096 --blocks 1048576 --ragged --rounds 11 >> $o 2>&1
echo "== crc mix" >> $o; timeout -k 10 120 python microbench/ab.py $A --kind crc32c --mixed --blocks 262144 --rounds 15 >> $o 2>&1
echo "== ragged 1K" >> $o; timeout -k 10 120 python microbench/ab.py $A --kind crc32c --block 1024 --blocks 2097152 --ragged --rounds 11 >> $o 2>&1
for v in 1 0; do
  cp microbench/mb_lib_ah$v.so speedb_amd/libspeedb_amd.so
  for w in sst walwrite; do
    echo "== $w ahead=$v" >> $o; timeout -k 10 180 python bench.py --workload $w --cpu-seconds 0 >> $o 2>&1
  done
done
cp microbench/mb_lib_ah1.so speedb_amd/libspeedb_amd.so
cat $o

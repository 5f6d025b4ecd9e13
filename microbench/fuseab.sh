# fused head mini round (generic CRC driver): parity, then A/B vs not fused
set -e
mkdir -p gpurun_out
o=gpurun_out/fuseab.log
: > $o
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/fu_pytest.log 2>&1 || { tail -40 gpurun_out/fu_pytest.log; exit 1; }
tail -2 gpurun_out/fu_pytest.log >> $o
A="microbench/mb_lib_fuse0.so microbench/mb_lib_fuse1.so"
echo "== crc mix" >> $o; timeout -k 10 120 python microbench/ab.py $A --kind crc32c --mixed --blocks 262144 --rounds 15 >> $o 2>&1
echo "== crc mix nojitter" >> $o; timeout -k 10 120 python microbench/ab.py $A --kind crc32c --mixed --nojitter --blocks 262144 --rounds 15 >> $o 2>&1
for v in 1 0; do
  cp microbench/mb_lib_fuse$v.so speedb_amd/libspeedb_amd.so
  for w in blob sst; do
    echo "== $w fuse=$v" >> $o; timeout -k 10 180 python bench.py --workload $w --cpu-seconds 0 >> $o 2>&1
  done
done
cp microbench/mb_lib_fuse1.so speedb_amd/libspeedb_amd.so
cat $o

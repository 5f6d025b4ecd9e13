# row transpose (permlane swaps) vs quad transpose (DPP) for the uniform CRC path
set -e
mkdir -p gpurun_out
o=gpurun_out/rtab.log
: > $o
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/rt_pytest.log 2>&1 || { tail -40 gpurun_out/rt_pytest.log; exit 1; }
tail -2 gpurun_out/rt_pytest.log >> $o
A="microbench/mb_lib_rt0.so microbench/mb_lib_rt1.so"
for b in 4096 65536; do
  n=$(( (1 << 32) / b ))
  echo "== uniform $b" >> $o; timeout -k 10 120 python microbench/ab.py $A --kind crc32c --block $b --blocks $n --rounds 15 >> $o 2>&1
done
for v in 1 0 1 0; do
  cp microbench/mb_lib_rt$v.so speedb_amd/libspeedb_amd.so
  echo "== bench crc32c rowt=$v" >> $o; timeout -k 10 180 python bench.py --cpu-seconds 0 >> $o 2>&1
done
cp microbench/mb_lib_rt1.so speedb_amd/libspeedb_amd.so
cat $o

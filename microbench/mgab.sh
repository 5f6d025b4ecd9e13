# mini groups (four small spans per iteration): parity, then A/B
set -e
mkdir -p gpurun_out
o=gpurun_out/mgab.log
: > $o
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/mg_pytest.log 2>&1 || { tail -40 gpurun_out/mg_pytest.log; exit 1; }
tail -2 gpurun_out/mg_pytest.log >> $o
timeout -k 10 200 python microbench/fusediag.py 2048 >> $o 2>&1
A="microbench/mb_lib_mg0.so microbench/mb_lib_mg1.so"
for b in 128 512 1000 4096; do
  n=$(( (1 << 29) / b ))
  echo "== ragged $b" >> $o; timeout -k 10 120 python microbench/ab.py $A --kind crc32c --block $b --blocks $n --ragged --rounds 7 >> $o 2>&1
done
echo "== crc mix" >> $o; timeout -k 10 120 python microbench/ab.py $A --kind crc32c --mixed --blocks 262144 --rounds 11 >> $o 2>&1
echo "== ragged 64K" >> $o; timeout -k 10 120 python microbench/ab.py $A --kind crc32c --block 65536 --blocks 16384 --ragged --rounds 7 >> $o 2>&1
for v in 1 0; do
  cp microbench/mb_lib_mg$v.so speedb_amd/libspeedb_amd.so
  echo "== walwrite mg=$v" >> $o; timeout -k 10 180 python bench.py --workload walwrite --cpu-seconds 0 >> $o 2>&1
done
cp microbench/mb_lib_mg1.so speedb_amd/libspeedb_amd.so
cat $o

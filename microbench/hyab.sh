# XXH3 hybrid (long spans on waves, short on rows): parity, then A/B
set -e
mkdir -p gpurun_out
o=gpurun_out/hyab.log
: > $o
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/hy_pytest.log 2>&1 || { tail -40 gpurun_out/hy_pytest.log; exit 1; }
tail -2 gpurun_out/hy_pytest.log >> $o
timeout -k 10 100 python microbench/x3diag.py >> $o 2>&1
A="microbench/mb_lib_hy0.so microbench/mb_lib_hy1.so"
echo "== xxh3 mix" >> $o; timeout -k 10 120 python microbench/ab.py $A --kind xxh3 --mixed --blocks 262144 --rounds 15 >> $o 2>&1
echo "== xxh3 mix nojitter" >> $o; timeout -k 10 120 python microbench/ab.py $A --kind xxh3 --mixed --nojitter --blocks 262144 --rounds 15 >> $o 2>&1
echo "== xxh3 ragged 4K" >> $o; timeout -k 10 120 python microbench/ab.py $A --kind xxh3 --block 4096 --blocks 262144 --ragged --rounds 11 >> $o 2>&1
for v in 1 0; do
  cp microbench/mb_lib_hy$v.so speedb_amd/libspeedb_amd.so
  echo "== sst hybrid=$v" >> $o; timeout -k 10 180 python bench.py --workload sst --cpu-seconds 0 >> $o 2>&1
done
cp microbench/mb_lib_hy1.so speedb_amd/libspeedb_amd.so
cat $o

# row-transposed loads in the generic driver (default now) and WAL verify (A/B)
set -e
mkdir -p gpurun_out
o=gpurun_out/wtab.log
: > $o
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/wt_pytest.log 2>&1 || { tail -40 gpurun_out/wt_pytest.log; exit 1; }
tail -2 gpurun_out/wt_pytest.log >> $o
timeout -k 10 100 python microbench/blobdiag.py 1048576 2048 >> $o 2>&1
timeout -k 10 200 python microbench/fusediag.py 2048 >> $o 2>&1
echo "== ab wal" >> $o; timeout -k 10 120 python microbench/ab.py microbench/mb_lib_wt0.so microbench/mb_lib_wt1.so --kind wal --blocks 131072 --rounds 15 >> $o 2>&1
for v in 1 0; do
  cp microbench/mb_lib_wt$v.so speedb_amd/libspeedb_amd.so
  echo "== bench wal wt=$v" >> $o; timeout -k 10 180 python bench.py --workload wal --cpu-seconds 0 >> $o 2>&1
done
cp microbench/mb_lib_wt1.so speedb_amd/libspeedb_amd.so
echo "== bench walwrite" >> $o; timeout -k 10 180 python bench.py --workload walwrite --cpu-seconds 0 >> $o 2>&1
cat $o

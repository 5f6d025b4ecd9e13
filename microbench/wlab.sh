# WAL verify: header prefetch + transposed loads, parity then A/B
set -e
mkdir -p gpurun_out
o=gpurun_out/wlab.log
: > $o
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/wl_pytest.log 2>&1 || { tail -40 gpurun_out/wl_pytest.log; exit 1; }
tail -2 gpurun_out/wl_pytest.log >> $o
echo "== ab wal (al1 = before, w1 = now)" >> $o; timeout -k 10 120 python microbench/ab.py microbench/mb_lib_al1.so microbench/mb_lib_w1.so --kind wal --blocks 131072 --rounds 15 >> $o 2>&1
for v in 1 0 1; do
  echo "== bench wal layout=$v" >> $o; MCK_CRC_LAYOUT=$v timeout -k 10 180 python bench.py --workload wal --cpu-seconds 0 >> $o 2>&1
done
cat $o

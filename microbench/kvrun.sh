set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/kv_pytest.log 2>&1
for v in kv1 kv0 kv1 kv0; do
  cp microbench/mb_lib_$v.so speedb_amd/libspeedb_amd.so
  echo "== $v" >> gpurun_out/kv_bench.log
  timeout -k 10 120 python bench.py --workload kv >> gpurun_out/kv_bench.log 2>&1
done
cp microbench/mb_lib_kv1.so speedb_amd/libspeedb_amd.so
tail -3 gpurun_out/kv_pytest.log; grep -E "==|frac" gpurun_out/kv_bench.log | sed 's/.*"roofline"/roofline/' | cut -c1-200

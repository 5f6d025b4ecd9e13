# WAL writer copy: non-temporal body stores (A/B by library swap), parity on the nt build
set -e
mkdir -p gpurun_out/nt
o=gpurun_out/nt/ntab.log
: > $o
cp speedb_amd/libspeedb_amd.so /tmp/lib_cur.so
for v in cur ntst cur ntst; do
  if [ $v = cur ]; then cp /tmp/lib_cur.so speedb_amd/libspeedb_amd.so; else cp microbench/mb_lib_$v.so speedb_amd/libspeedb_amd.so; fi
  echo "== $v" >> $o; timeout -k 10 180 python bench.py --workload walwrite --cpu-seconds 0 >> $o 2>&1
done
timeout -k 10 300 python -u -m pytest tests/test_wal_writer.py -m gpu -x -q --timeout 120 --timeout-method thread >> $o 2>&1
cp /tmp/lib_cur.so speedb_amd/libspeedb_amd.so
cat $o

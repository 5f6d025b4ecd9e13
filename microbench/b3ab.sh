# v_bitop3 XOR-3 in the CRC table steps: parity, then A/B
set -e
mkdir -p gpurun_out
o=gpurun_out/b3ab.log
: > $o
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/b3_pytest.log 2>&1 || { tail -40 gpurun_out/b3_pytest.log; exit 1; }
tail -2 gpurun_out/b3_pytest.log >> $o
timeout -k 10 100 python microbench/blobdiag.py 1048576 2048 >> $o 2>&1
A="microbench/mb_lib_b0.so microbench/mb_lib_b3.so"
echo "== uniform 4K" >> $o; timeout -k 10 120 python microbench/ab.py $A --kind crc32c --rounds 15 >> $o 2>&1
echo "== crc mix" >> $o; timeout -k 10 120 python microbench/ab.py $A --kind crc32c --mixed --blocks 262144 --rounds 15 >> $o 2>&1
echo "== wal" >> $o; timeout -k 10 120 python microbench/ab.py $A --kind wal --blocks 131072 --rounds 15 >> $o 2>&1
for v in 3 0; do
  cp microbench/mb_lib_b$v.so speedb_amd/libspeedb_amd.so
  for w in crc32c sst; do
    echo "== $w b=$v" >> $o; timeout -k 10 180 python bench.py --workload $w --cpu-seconds 0 >> $o 2>&1
  done
done
cp microbench/mb_lib_b3.so speedb_amd/libspeedb_amd.so
cat $o

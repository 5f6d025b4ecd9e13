# transposed-load generic CRC driver: parity, then A/B vs the chunk layout
set -e
mkdir -p gpurun_out
o=gpurun_out/tlab2.log
: > $o
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tl2_pytest.log 2>&1 || { tail -40 gpurun_out/tl2_pytest.log; exit 1; }
tail -2 gpurun_out/tl2_pytest.log >> $o
for w in sst blob walwrite; do
  for v in 1 0; do
    echo "== $w layout=$v" >> $o; MCK_CRC_LAYOUT=$v timeout -k 10 180 python bench.py --workload $w --cpu-seconds 0 >> $o 2>&1
  done
done
for v in 1 0; do
  echo "== crc mix layout=$v" >> $o; MCK_CRC_LAYOUT=$v timeout -k 10 120 python microbench/ab.py speedb_amd/libspeedb_amd.so --kind crc32c --mixed --blocks 262144 --rounds 15 >> $o 2>&1
done
cat $o

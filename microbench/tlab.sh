# transposed-load CRC (uniform whole-round spans): parity, then A/B vs the chunk layout
set -e
mkdir -p gpurun_out
o=gpurun_out/tlab.log
: > $o
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tl_pytest.log 2>&1 || { tail -40 gpurun_out/tl_pytest.log; exit 1; }
tail -2 gpurun_out/tl_pytest.log >> $o
for v in 1 0 1 0; do
  echo "== layout=$v" >> $o; MCK_CRC_LAYOUT=$v timeout -k 10 180 python bench.py --workload crc32c --cpu-seconds 0 >> $o 2>&1
done
echo "== file layout=1" >> $o; timeout -k 10 180 python bench.py --workload file --cpu-seconds 0 >> $o 2>&1
echo "== file layout=0" >> $o; MCK_CRC_LAYOUT=0 timeout -k 10 180 python bench.py --workload file --cpu-seconds 0 >> $o 2>&1
cat $o

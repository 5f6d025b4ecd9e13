# WAL writer: CRC/copy overlap pieces A/B (MCK_WAL_PIECES), after parity
set -e
mkdir -p gpurun_out/wp
o=gpurun_out/wp/wpab.log
: > $o
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/wp/pytest.log 2>&1 || { tail -40 gpurun_out/wp/pytest.log; exit 1; }
tail -2 gpurun_out/wp/pytest.log >> $o
for v in 1 2 4 8 4 1; do
  echo "== pieces $v" >> $o; MCK_WAL_PIECES=$v timeout -k 10 180 python bench.py --workload walwrite --cpu-seconds 0 >> $o 2>&1
done
cat $o

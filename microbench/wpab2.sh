# WAL writer: more, smaller pieces (copy reads of a piece still in the MALL?)
set -e
mkdir -p gpurun_out/wp2
o=gpurun_out/wp2/wpab.log
: > $o
for v in 8 16 32 64 8 32; do
  echo "== pieces $v" >> $o; MCK_WAL_PIECES=$v timeout -k 10 180 python bench.py --workload walwrite --cpu-seconds 0 >> $o 2>&1
done
cat $o

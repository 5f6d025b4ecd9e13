# WAL writer copy kernel variants: rocprof kernel averages per library
set -e
mkdir -p gpurun_out/wc2
o=gpurun_out/wc2/wcab.log
: > $o
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
cp speedb_amd/libspeedb_amd.so /tmp/lib_cur.so
for v in cur wc0 wcnt wc1 wc1nt wc0; do
  if [ $v = cur ]; then cp /tmp/lib_cur.so speedb_amd/libspeedb_amd.so; else cp microbench/mb_lib_$v.so speedb_amd/libspeedb_amd.so; fi
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/wc2/$v -o run --output-format csv -- python3 bench.py --workload walwrite --cpu-seconds 0 > gpurun_out/wc2/$v.txt 2>&1
  echo "== $v: $(grep -h k_wal_copy gpurun_out/wc2/$v/*kernel_stats.csv | cut -d, -f1-4 | head -1)" >> $o
done
cp /tmp/lib_cur.so speedb_amd/libspeedb_amd.so
cat $o

# WAL writer copy kernel: pipelined (new) vs per-loop (MCK_WAL_COPY_PIPE=0), parity then A/B
set -e
mkdir -p gpurun_out/wc
o=gpurun_out/wc/wcab.log
: > $o
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/wc/pytest.log 2>&1 || { tail -40 gpurun_out/wc/pytest.log; exit 1; }
tail -2 gpurun_out/wc/pytest.log >> $o
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/wc/new -o run -- python3 bench.py --workload walwrite --cpu-seconds 0 >> $o 2>&1
echo "== new done" >> $o
cp speedb_amd/libspeedb_amd.so /tmp/lib_new.so
cp microbench/mb_lib_wc0.so speedb_amd/libspeedb_amd.so
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/wc/old -o run -- python3 bench.py --workload walwrite --cpu-seconds 0 >> $o 2>&1
echo "== old done" >> $o
cp /tmp/lib_new.so speedb_amd/libspeedb_amd.so
timeout -k 10 180 python bench.py --workload walwrite --cpu-seconds 0 >> $o 2>&1
cat $o

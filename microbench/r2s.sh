set -e
mkdir -p gpurun_out/r2s
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2s/pytest_gpu.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r2s/smoke.log 2>&1
timeout -k 10 120 python bench.py --warmup 5 --steps 20 > gpurun_out/r2s/bench.json 2> gpurun_out/r2s/bench.err
for k in 1 2; do
timeout -k 10 120 python bench.py --workload walwrite > gpurun_out/r2s/ww_blk$k.json 2>/dev/null
MCK_WAL_ORDER=interleaved timeout -k 10 120 python bench.py --workload walwrite > gpurun_out/r2s/ww_ilv$k.json 2>/dev/null
done

set -o pipefail
OUT=gpurun_out/r2m
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver_shape.json 2> $OUT/bench.err || exit 1
cat $OUT/bench_driver_shape.json
WORKLOADS="crc32c walwrite sst" bash profiles/run_all.sh r2m > $OUT/run_all.log 2>&1 || { tail -20 $OUT/run_all.log; exit 1; }
tail -5 $OUT/run_all.log

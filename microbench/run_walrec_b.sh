set -uo pipefail
export TMPDIR=/tmp
o=gpurun_out/r6d
mkdir -p $o
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_wal_recover.py tests/test_wal_reader.py tests/test_wal_writer.py tests/test_cpp_mirror.py -m gpu > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -3 $o/tests.log
timeout -k 10 300 python3 bench.py --workload walrecover --walrec-shape full32k --steps 20 --warmup 10 > $o/full32k.json 2> $o/full32k.err || exit 1
timeout -k 10 400 python3 bench.py --workload walrecover --walrec-shape mix --steps 20 --warmup 10 > $o/mix.json 2> $o/mix.err || exit 1
echo ok

set -uo pipefail
export TMPDIR=/tmp
o=gpurun_out/r6f
mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wal_recover.py -m gpu > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
MCK_WALREC_U2=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wal_recover.py -m gpu > $o/tests_u2.log 2>&1 || { tail -30 $o/tests_u2.log; exit 1; }
for sh in full32k mix; do
  A="--workload walrecover --walrec-shape $sh --steps 20 --warmup 10 --cpu-seconds 0"
  timeout -k 10 300 python3 bench.py $A --no-verify > $o/$sh.json 2>&1 || exit 1
  MCK_WALREC_U2=1 timeout -k 10 300 python3 bench.py $A --no-verify > $o/${sh}_u2.json 2>&1 || exit 1
done
echo ok

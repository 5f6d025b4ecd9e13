#!/bin/bash
# WAL writer A/B: parity of the in-tree library, then
# per variant the walwrite bench (twice, interleaved) and a WRITE_SIZE pass.
#   $1 = output tag; WV = variants (_variants/<v>.so, "new" = in-tree)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-walwab}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_wal_writer.py tests/test_wal_reader.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
V=$PWD/microbench/_variants
run() {  # $1 = variant, rest = command
  local v=$1; shift
  if [ $v = new ]; then env -u SPEEDB_AMD_LIB "$@"; else env SPEEDB_AMD_AB=1 SPEEDB_AMD_LIB=$V/$v.so "$@"; fi
}
A="--workload walwrite --cpu-seconds 0 ${WARGS:-}"
for pass in 1 2; do
  for v in ${WV:-r5w0 new}; do
    run $v timeout -k 10 180 python -u bench.py $A --steps 20 --warmup 10 > $O/${v}_$pass.json || exit 1
  done
done
for v in ${WV:-r5w0 new}; do
  run $v timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_$v -o pmc --output-format csv \
    -- python3 bench.py $A --no-verify --steps 5 --warmup 2 > $O/pmcrun_$v.txt 2>&1 || exit 1
  python3 microbench/pmc_summary.py $O/pmc_$v k_wal_write_il > $O/write_$v.txt || exit 1
  echo "$v $(for p in 1 2; do python3 -c "import json; d=json.load(open('$O/${v}_$p.json')); print(d['roofline']['frac'], d['roofline']['kernel_avg_ms'], d['verified'], d['config'].get('stream_bytes'), end=' ')"; done) $(grep WRITE_SIZE $O/write_$v.txt)"
done

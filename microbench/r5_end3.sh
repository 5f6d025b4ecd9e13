#!/bin/bash
# Round-5 evidence after the XXH3 row loop's cache-policy change
# (profiles/r5/x3_align/) and the 8-lane row loop unroll
# (profiles/r5/rows_pace/): default bench lines of the workloads whose
# kernels changed, then kernel traces + FETCH/WRITE passes for per-KV
# protection and block KV (1000-B and 100-B values).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
tag=r5end3
O=gpurun_out/bench_$tag
mkdir -p $O
B="timeout -k 10 240 python -u bench.py"
$B --workload kv > $O/kv.json || exit 1
$B --workload blockkv > $O/blockkv.json || exit 1
$B --workload blockkv --kv-value-bytes 100 --cpu-seconds 0 > $O/blockkv100.json || exit 1
$B --workload walrec --cpu-seconds 0 > $O/walrec.json || exit 1
$B --workload crc32c > $O/crc32c.json || exit 1
bash profiles/run_profile.sh $tag kv || exit 1
bash profiles/run_profile.sh $tag blockkv || exit 1
bash profiles/run_profile.sh ${tag}_100 blockkv --kv-value-bytes 100 || exit 1
echo "end3 done"

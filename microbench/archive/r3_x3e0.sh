#!/bin/bash
# round 3: XXH3 rows driver takes the dword before a segment from registers
# (no re-read of the previous segment's last line) -- parity, rate, traffic
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r3x3}
O=gpurun_out/$T
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_block_protection.py tests/test_sst_file.py tests/test_handoff.py tests/test_cpp_mirror.py -k "not subprocess" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="timeout -k 10 180 python -u bench.py --cpu-seconds 0"
H="env SPEEDB_AMD_LIB=$PWD/microbench/_variants/head.so"
for k in 1 2; do
  $B --workload xxh3 > $O/xxh3_new$k.json || exit 1
  $H $B --workload xxh3 > $O/xxh3_head$k.json || exit 1
done
$B --workload kv > $O/kv_new.json || exit 1
$H $B --workload kv > $O/kv_head.json || exit 1
$B --workload sst --sst-types xxh3 > $O/sstx_new.json || exit 1
$H $B --workload sst --sst-types xxh3 > $O/sstx_head.json || exit 1
for f in $O/*.json; do echo "$f $(python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['roofline']['frac'], d['roofline'].get('kernel_avg_ms'))")"; done
timeout -k 10 400 bash profiles/run_profile.sh $T xxh3 || exit 1
timeout -k 10 400 bash profiles/run_profile.sh $T kv || exit 1
python3 -c "import json; [print(w, json.load(open('gpurun_out/prof_${T}_'+w+'/traffic.json'))['traffic_over_alg']) for w in ('xxh3','kv')]"

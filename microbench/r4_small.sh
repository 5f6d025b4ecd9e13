#!/bin/bash
# round 4: the small-batch wave-per-span path -- parity (default and forced)
# then the latency line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/${1:-small}
mkdir -p $O
T="timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread"
$T tests/test_gpu_parity.py tests/test_sst_file.py tests/test_blob_file.py tests/test_wal_reader.py "tests/test_crc_rows.py::test_auto_kernel_forced_drivers_subprocess[small]" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u bench.py --workload latency > $O/latency.json || exit 1
python3 -c "import json; d=json.load(open('$O/latency.json')); [print(r) for r in d['rows']]; print(d['crossover_blocks_device_resident'], d['crossover_blocks_pinned'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/lat_trace -o t --output-format csv -- python3 bench.py --workload latency > $O/lat_trace.txt 2>&1 || exit 1
python3 - $O/lat_trace <<'PY'
import csv,glob,sys
for f in glob.glob(sys.argv[1]+'/**/*kernel_stats.csv',recursive=True):
    for r in csv.DictReader(open(f)):
        print(r['Name'][:80], r['Calls'], r['AverageNs'])
PY

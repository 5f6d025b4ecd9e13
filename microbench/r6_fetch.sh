#!/bin/bash
# One FETCH_SIZE + WRITE_SIZE pass (kernel trace only) of a bench command:
#   TAG=<dir> NAME=<name> bash microbench/r6_fetch.sh <bench args>
# -> gpurun_out/$TAG/$NAME/{pmc_fetch,pmc_write}/ + a summary line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
o=gpurun_out/${TAG:-r6_fetch}/${NAME:-run}
mkdir -p $o
A="--cpu-seconds 0 --no-verify --steps 10 --warmup 3 --settle-ms 50 $*"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $o/pmc_fetch -o pmc --output-format csv -- python3 bench.py $A > $o/bench_fetch.txt 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $o/pmc_write -o pmc --output-format csv -- python3 bench.py $A > $o/bench_write.txt 2>&1 || exit 1
python3 - $o <<'PY'
import csv, json, sys, collections
o = sys.argv[1]
line = [json.loads(l) for l in open(o + "/bench_fetch.txt") if l.startswith("{")][0]
alg = line["roofline"]["alg_bytes_per_launch"]
def per_kernel(path, ctr):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == ctr:
            d[r["Kernel_Name"][:60]].append(float(r["Counter_Value"]) * 1024)
    return {k: sum(v) / len(v) for k, v in d.items()}
f = per_kernel(o + "/pmc_fetch/pmc_counter_collection.csv", "FETCH_SIZE")
w = per_kernel(o + "/pmc_write/pmc_counter_collection.csv", "WRITE_SIZE")
for k in f:
    print(f"{k:60s} fetch x2 {2*f[k]/alg:.4f}  write {w.get(k, 0)/alg:.4f} of alg {alg}")
PY

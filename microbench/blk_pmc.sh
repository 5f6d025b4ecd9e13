#!/bin/bash
# Block KV (100-B values): available TA/TCP/TCC counters, then one pass of them.
out=gpurun_out/$1
mkdir -p $out
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $out/avail.txt 2>&1 || true
grep -o -E "\b(TA|TCP|TCC)_[A-Z0-9_]+(_sum)?\b" $out/avail.txt | sort -u > $out/names.txt || true
timeout -s KILL 90 rocprofv3 --pmc ${PMC:-TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE} --kernel-trace -d $out/p1 -o pmc --output-format csv -- python3 bench.py --workload blockkv --kv-value-bytes 100 --steps 2 --warmup 1 --settle-ms 0 --no-verify > $out/p1.txt 2>&1 || { tail -5 $out/p1.txt; exit 1; }
python3 - $out <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for f in glob.glob(out + "/p1/**/*counter_collection.csv", recursive=True):
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:28]
        if "k_block" not in k: continue
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[(k, r["Counter_Name"])] += 1
    for k, d in acc.items():
        print(k, {c: f"{v / n[(k, c)]:.4g}" for c, v in d.items()})
PY

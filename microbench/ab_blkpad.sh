#!/bin/bash
# Block KV walk occupancy A/B: product (2 workgroups per CU) vs a variant
# padded to 1 workgroup per CU; time and per-kernel FETCH_SIZE.
set -uo pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/r6c_blkpad
mkdir -p $o
V=microbench/_variants/blkpad1.so
for vb in 100 1000; do
  A="--workload blockkv --kv-value-bytes $vb --steps 20 --warmup 5 --cpu-seconds 0"
  timeout -k 10 200 python3 bench.py $A > $o/base_$vb.json 2>&1 || exit 1
  timeout -k 10 200 python3 bench.py $A --engine-lib $V > $o/pad_$vb.json 2>&1 || exit 1
  timeout -k 10 200 python3 bench.py $A > $o/base2_$vb.json 2>&1 || exit 1
done
for t in base pad; do
  E=""; [ $t = pad ] && E="--engine-lib $V"
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $o/f_$t -o pmc --output-format csv -- python3 bench.py --workload blockkv --kv-value-bytes 100 --steps 2 --warmup 1 --settle-ms 0 --no-verify --cpu-seconds 0 $E > $o/f_$t.txt 2>&1 || { tail -5 $o/f_$t.txt; exit 1; }
done
python3 - $o <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for t in ("base", "pad"):
    for f in glob.glob(f"{out}/f_{t}/**/*counter_collection.csv", recursive=True):
        acc = collections.defaultdict(float); n = collections.Counter()
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"][:30]
            if "k_block" not in k: continue
            acc[k] += float(r["Counter_Value"]); n[k] += 1
        for k, v in acc.items():
            print(t, k, f"FETCH x1024x2 per launch = {v / n[k] * 2048 / 1e9:.3f} GB")
PY
echo ok

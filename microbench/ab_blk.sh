#!/bin/bash
# Block KV walk A/B: product vs variant libraries (VARS="name ..."), time
# (100-B and 1000-B values) and per-kernel FETCH_SIZE / WRITE_SIZE at 100-B.
set -uo pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/${OUT:-r6c_blk}
mkdir -p $o
for vb in 100 1000; do
  A="--workload blockkv --kv-value-bytes $vb --steps 20 --warmup 5 --cpu-seconds 0"
  timeout -k 10 200 python3 bench.py $A > $o/base_$vb.json 2>&1 || exit 1
  for v in $VARS; do
    timeout -k 10 200 python3 bench.py $A --engine-lib microbench/_variants/$v.so > $o/${v}_$vb.json 2>&1 || exit 1
  done
done
for t in base $VARS; do
  E=""; [ $t != base ] && E="--engine-lib microbench/_variants/$t.so"
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace -d $o/${c}_$t -o pmc --output-format csv -- python3 bench.py --workload blockkv --kv-value-bytes 100 --steps 2 --warmup 1 --settle-ms 0 --no-verify --cpu-seconds 0 $E > $o/${c}_$t.txt 2>&1 || { tail -5 $o/${c}_$t.txt; exit 1; }
  done
done
python3 - $o base $VARS <<'PY'
import csv, glob, sys, collections, json
out = sys.argv[1]
for t in sys.argv[2:]:
    for vb in (100, 1000):
        d = json.loads(open(f"{out}/{t}_{vb}.json").read().strip().splitlines()[-1])
        print(t, vb, d["ms_per_step"], d["roofline"]["frac"])
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        for f in glob.glob(f"{out}/{c}_{t}/**/*counter_collection.csv", recursive=True):
            acc = collections.defaultdict(float); n = collections.Counter()
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"][:30]
                if "k_block" not in k: continue
                acc[k] += float(r["Counter_Value"]); n[k] += 1
            for k, v in acc.items():
                print(" ", t, c, k, f"{v / n[k] * 1024 * (2 if c == 'FETCH_SIZE' else 1) / 1e9:.3f} GB per launch")
PY
echo ok

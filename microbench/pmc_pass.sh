#!/bin/bash
# One --pmc pass per counter set over a bench workload; per-kernel averages.
#   $1 = out tag, $2 = kernel-name substring, rest = bench args
# PMC1, PMC2, ... = counter sets (one rocprofv3 run each)
out=gpurun_out/$1; ksub=$2; shift 2
mkdir -p $out
export TMPDIR=/tmp
i=0
for set in "$PMC1" "$PMC2" "$PMC3" "$PMC4"; do
  [ -z "$set" ] && continue
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace -d $out/p$i -o pmc --output-format csv -- python3 bench.py "$@" --steps 2 --warmup 1 --settle-ms 0 --no-verify --cpu-seconds 0 > $out/p$i.txt 2>&1 || { tail -5 $out/p$i.txt; exit 1; }
done
python3 - $out "$ksub" <<'PY'
import csv, glob, sys, collections
out, ksub = sys.argv[1], sys.argv[2]
for f in sorted(glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if ksub not in k: continue
        k = k[:40]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[(k, r["Counter_Name"])] += 1
    for k, d in acc.items():
        print(k, {c: f"{v / n[(k, c)]:.4g}" for c, v in d.items()})
PY

#!/bin/bash
# EXPERIMENT: block KV walk traffic vs occupancy
# (historical: the MCK_PAD_* hooks this sweep set were replaced by the fixed
# kBlkLayoutLdsPad / kBlkWalkLdsPad in mck_engine.hip; results in profiles/r4/blockkv_occupancy)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/kvfetch
mkdir -p $O
A="--workload blockkv --kv-value-bytes ${KV_BYTES:-100} --cpu-seconds 0 --no-verify --steps 3 --warmup 2"
for cfg in ${PAD_CFGS:-0:0}; do
  l=${cfg%%:*}; k=${cfg##*:}
  MCK_PAD_LAYOUT=$l MCK_PAD_KV=$k timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/f_${l}_$k -o p --output-format csv -- python3 bench.py $A > $O/b_${l}_$k.txt 2>&1 || exit 1
  python3 - $O/f_${l}_$k <<'PY'
import csv,glob,sys,collections
agg=collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1]+'/**/*counter_collection.csv',recursive=True):
    for r in csv.DictReader(open(f)):
        if 'block' in r['Kernel_Name']: agg[r['Kernel_Name'].split('(')[0][-28:]][r['Counter_Name']].append(float(r['Counter_Value']))
for k,v in agg.items(): print(sys.argv[1].split('/')[-1], k, {c: round(sum(x)/len(x)) for c,x in v.items()})
PY
done

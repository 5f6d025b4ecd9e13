#!/bin/bash
# EXPERIMENT: block KV walk occupancy (LDS padding) vs time
# (historical: the MCK_PAD_* hooks this sweep set were replaced by the fixed
# kBlkLayoutLdsPad / kBlkWalkLdsPad in mck_engine.hip; results in profiles/r4/blockkv_occupancy)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/kvpad
mkdir -p $O
A="--workload blockkv --kv-value-bytes ${KV_BYTES:-100} --cpu-seconds 0 --no-verify --steps 5 --warmup 3"
for cfg in ${PAD_CFGS:-0:0}; do
  l=${cfg%%:*}; k=${cfg##*:}
  MCK_PAD_LAYOUT=$l MCK_PAD_KV=$k timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/t_${l}_$k -o t --output-format csv -- python3 bench.py $A > $O/b_${l}_$k.txt 2>&1 || exit 1
  python3 - $O/t_${l}_$k <<'PY'
import csv,glob,sys
for f in glob.glob(sys.argv[1]+'/**/*kernel_stats.csv',recursive=True):
    for r in csv.DictReader(open(f)):
        if 'block' in r['Name']: print(sys.argv[1].split('/')[-1], r['Name'].split('(')[0][-30:], round(float(r['AverageNs'])/1000,1))
PY
done

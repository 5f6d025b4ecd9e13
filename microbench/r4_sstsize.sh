#!/bin/bash
# round 4: SST image kernel time vs image size (the fixed per-launch tail)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/sstsize
mkdir -p $O
for t in xxh3 crc32c; do
  for g in 1 2 4; do
    timeout -k 10 240 python -u bench.py --workload sst --sst-types $t --sst-bytes $((g << 30)) --cpu-seconds 0 --steps 20 --warmup 10 > $O/${t}_$g.json || exit 1
    echo "$t $g $(python3 -c "import json; d=json.load(open('$O/${t}_$g.json')); print(d['roofline']['frac'], d['roofline']['kernel_avg_ms'])")"
  done
done

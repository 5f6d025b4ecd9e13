#!/bin/bash
# Round profile of every bench workload on the GPU box (run from the repo
# root via gpurun): bench lines (default flags) + rocprofv3 kernel trace/stats
# and FETCH_SIZE/WRITE_SIZE passes per workload.  $1 = tag.
set -euo pipefail
tag=${1:-run}
shift || true
wls=${WORKLOADS:-"crc32c xxh3 sst wal file kv walwrite blob host"}
mkdir -p gpurun_out/bench_$tag
for wl in $wls; do
  cpu=0
  [ "$wl" = crc32c ] && cpu=12
  [ "$wl" = xxh3 ] && cpu=6
  timeout -k 10 240 python bench.py --workload $wl --cpu-seconds $cpu > gpurun_out/bench_$tag/$wl.json 2> gpurun_out/bench_$tag/$wl.err
  echo "bench $wl done"
  if [ "$wl" != host ]; then
    bash profiles/run_profile.sh $tag $wl
  fi
done

#!/bin/bash
# Round-5 end-of-round evidence on the GPU box: default-flag bench lines,
# then rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE (+ SQ counters where
# PROFILE_SQ) per workload via profiles/run_profile.sh, and the WAL verify
# FETCH calibration (request counts next to FETCH_SIZE).
#   $1 = part (1: bench lines, 2: profiles A, 3: profiles B + calibration)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
tag=${R5_TAG:-r5end}
O=gpurun_out/bench_$tag
mkdir -p $O
B="timeout -k 10 240 python -u bench.py"
case "${1:-1}" in
1)
  $B --workload crc32c > $O/crc32c.json || exit 1
  for wl in xxh3 sst wal file kv walwrite blob blockkv walrec; do
    $B --workload $wl --cpu-seconds 0 > $O/$wl.json || exit 1
  done
  $B --workload blockkv --kv-value-bytes 100 --cpu-seconds 0 > $O/blockkv100.json || exit 1
  $B --workload crc32c --block-bytes 4300 --blocks 1000000 --cpu-seconds 0 > $O/u4300.json || exit 1
  $B --workload ragged --span-min 4100 --span-max 4400 --span-bytes $((4 << 30)) --cpu-seconds 0 > $O/r4100.json || exit 1
  $B --workload ragged --span-min 4096 --span-max 4096 --span-bytes $((4 << 30)) --cpu-seconds 0 > $O/r4096.json || exit 1
  $B --workload ragged --span-min 100 --span-max 300 --cpu-seconds 0 > $O/r100.json || exit 1
  ;;
2)
  PROFILE_SQ=1 bash profiles/run_profile.sh $tag crc32c || exit 1
  PROFILE_SQ=1 bash profiles/run_profile.sh $tag sst || exit 1
  PROFILE_SQ=1 bash profiles/run_profile.sh ${tag}_u4300 crc32c --block-bytes 4300 --blocks 1000000 || exit 1
  PROFILE_SQ=1 bash profiles/run_profile.sh ${tag}_r4100 ragged --span-min 4100 --span-max 4400 --span-bytes $((4 << 30)) || exit 1
  PROFILE_SQ=1 bash profiles/run_profile.sh $tag walrec || exit 1
  ;;
3)
  for wl in wal walwrite blob blockkv kv xxh3 file; do
    bash profiles/run_profile.sh $tag $wl || exit 1
  done
  bash profiles/run_profile.sh ${tag}_100 blockkv --kv-value-bytes 100 || exit 1
  PROFILE_SQ=1 bash profiles/run_profile.sh ${tag}_r100 ragged --span-min 100 --span-max 300 || exit 1
  # WAL verify FETCH calibration: the bench image reads every byte once
  # (one kFullType record per 32 KiB block); request counts beside FETCH_SIZE
  d=gpurun_out/prof_${tag}_wal
  timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --kernel-trace -d $d/pmc_req -o pmc \
    --output-format csv -- python3 bench.py --workload wal --cpu-seconds 0 --no-verify > $d/bench_req.txt 2>&1 || exit 1
  ;;
esac
echo "part ${1:-1} done"

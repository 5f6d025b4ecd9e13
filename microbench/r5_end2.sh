#!/bin/bash
# Round-5 evidence after the driver-choice changes (uniform CRC on k_crc_ragged,
# uniform XXH3 >= 3 KiB on the wave kernel, row thresholds): every default
# bench line again, then kernel traces + FETCH/WRITE passes for the workloads
# whose kernel changed (crc32c, file, xxh3).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
R5_TAG=r5end2 bash microbench/r5_end.sh 1 || exit 1
PROFILE_SQ=1 bash profiles/run_profile.sh r5end2 crc32c || exit 1
bash profiles/run_profile.sh r5end2 file || exit 1
bash profiles/run_profile.sh r5end2 xxh3 || exit 1
echo "end2 done"

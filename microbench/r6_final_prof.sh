#!/bin/bash
# Round-6 end state, part B: kernel traces + FETCH/WRITE passes -> the
# tracked traffic files (profiles/traffic_<shape>.json via run_profile.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
tag=${TAG:-r6final}
bash profiles/run_profile.sh $tag crc32c || exit 1
bash profiles/run_profile.sh $tag sst || exit 1
TRAFFIC_NAME=walrecover_full32k bash profiles/run_profile.sh ${tag}_full32k walrecover --walrec-shape full32k || exit 1
TRAFFIC_NAME=walrecover_mix bash profiles/run_profile.sh ${tag}_mix walrecover --walrec-shape mix || exit 1
TRAFFIC_NAME=r100_ragged_xxh3 bash profiles/run_profile.sh ${tag}_x3r100 ragged --ragged-hash xxh3 --span-min 100 --span-max 300 || exit 1
echo "final B done"

#!/bin/bash
# Round-6 same-box A/B: the in-tree engine ("new") vs the builds
# microbench/_variants/<name>.so listed in $VARIANTS (default: $BASE) on the
# workloads named in $WL ("name|bench args" entries separated by ';'),
# interleaved, twice each.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/${TAG:-r6_ab}
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $TESTS > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
IFS=';' read -ra ITEMS <<< "$WL"
for it in "${ITEMS[@]}"; do
  name=${it%%|*}; args=${it#*|}
  VS="new ${VARIANTS:-${BASE%.so}}"
  for v in $VS $VS; do
    if [ $v = new ]; then E=""; else E="--engine-lib microbench/_variants/$v.so"; fi
    timeout -k 10 240 python -u bench.py --cpu-seconds 0 --no-verify $args $E >> $O/${name}_$v.json || exit 1
  done
done
python3 - "$O" <<'PY'
import json, sys, glob, os, collections
r = collections.defaultdict(list)
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            r[os.path.basename(f)[:-5]].append(d["roofline"]["frac"])
for k, v in sorted(r.items()):
    print(f"{k:28s} " + " ".join(f"{x:.4f}" for x in v) + f"   max {max(v):.4f}")
PY
echo done

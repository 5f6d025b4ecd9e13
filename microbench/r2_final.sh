#!/bin/bash
# Round-end check: full GPU suite, smoke, the driver's bench command, walwrite.
set -o pipefail
OUT=gpurun_out/${1:-r2final}
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit 1
tail -1 $OUT/smoke.log
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit 1
python -c "import json; d=json.load(open('$OUT/bench.json')); print('headline', d['value'], d['roofline']['frac'], d['cpu_baseline']['value'])"
timeout -k 10 120 python bench.py --workload walwrite --cpu-seconds 0 > $OUT/walwrite.json 2>> $OUT/bench.err || exit 1
python -c "import json; d=json.load(open('$OUT/walwrite.json')); print('walwrite', d['value'], d['roofline']['frac'], d['roofline'].get('traffic'))"

#!/bin/bash
# round 3: unit-stream driver vs the 4 KiB-round wave driver: rates and SQ
# instruction mix on uniform 4300-B blocks (parity first)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r3u2}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_crc_units.py tests/test_block_protection.py tests/test_gpu_parity.py -k "units or xxh3 or large_ragged or sst or block or xxph3" > $O/units_tests.log 2>&1 || { tail -30 $O/units_tests.log; exit 1; }
tail -2 $O/units_tests.log
B="timeout -k 10 180 python -u bench.py --steps 20 --warmup 20 --cpu-seconds 0"
for d in units wave; do
  $B --crc-driver $d --workload crc32c --block-bytes 4300 --blocks 1000000 > $O/u4300_$d.json || exit 1
  $B --crc-driver $d --workload ragged --span-min 4100 --span-max 4400 --span-bytes $((4<<30)) > $O/r4100_$d.json || exit 1
  $B --crc-driver $d --workload ragged --span-min 4096 --span-max 4096 --span-bytes $((4<<30)) > $O/r4096_$d.json || exit 1
  $B --crc-driver $d --workload sst --sst-types crc32c --sst-bytes $((1<<30)) > $O/sst1g_$d.json || exit 1
done
TK="env SPEEDB_AMD_LIB=$PWD/microbench/_variants/units_ticket.so"
$TK $B --crc-driver units --workload crc32c --block-bytes 4300 --blocks 1000000 > $O/u4300_ticket.json || exit 1
$TK $B --crc-driver units --workload ragged --span-min 4100 --span-max 4400 --span-bytes $((4<<30)) > $O/r4100_ticket.json || exit 1
$TK $B --workload sst --sst-bytes $((1<<30)) > $O/sst1g_both_old.json || exit 1
$B --workload sst --sst-types xxh3 --sst-bytes $((1<<30)) > $O/sst1g_x3.json || exit 1
$B --workload sst --sst-bytes $((1<<30)) > $O/sst1g_both.json || exit 1
$B --workload blockkv --kv-value-bytes 1000 > $O/blk1000.json || exit 1
$B --workload blockkv --kv-value-bytes 100 > $O/blk100.json || exit 1
for f in $O/*.json; do echo "$f $(python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['roofline']['frac'], d['roofline']['kernel_avg_ms'], d['verified'])")"; done
for d in units wave; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --kernel-trace -d $O/pmc_$d -o pmc --output-format csv -- python3 bench.py --crc-driver $d --workload crc32c --block-bytes 4300 --blocks 1000000 --steps 2 --warmup 1 --settle-ms 0 --no-verify --cpu-seconds 0 > $O/pmc_$d.txt 2>&1 || { tail -5 $O/pmc_$d.txt; exit 1; }
done
python3 - $O <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
for d in ("units", "wave"):
    acc = collections.defaultdict(float); n = collections.Counter()
    for f in glob.glob(f"{O}/pmc_{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "crc_auto" not in r["Kernel_Name"]: continue
            acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    print(d, {c: f"{v / n[c]:.4g}" for c, v in sorted(acc.items())})
PY
# nt FETCH_SIZE / WRITE_SIZE calibration on known byte counts (4 GiB per launch)
timeout -k 10 60 ./microbench/nt_calib > $O/nt_calib.txt 2>&1 || { cat $O/nt_calib.txt; exit 1; }
cat $O/nt_calib.txt
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/nt_fetch -o pmc --output-format csv -- ./microbench/nt_calib > $O/nt_fetch.txt 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/nt_write -o pmc --output-format csv -- ./microbench/nt_calib > $O/nt_write.txt 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --kernel-trace -d $O/nt_req -o pmc --output-format csv -- ./microbench/nt_calib > $O/nt_req.txt 2>&1 || echo "req counters failed"
python3 - $O <<'PY'
import csv, glob, sys
O = sys.argv[1]
for d in ("nt_fetch", "nt_write", "nt_req"):
    for f in glob.glob(f"{O}/{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            print(d, r["Dispatch_Id"], r["Kernel_Name"][:40], r["Counter_Name"], r["Counter_Value"])
PY

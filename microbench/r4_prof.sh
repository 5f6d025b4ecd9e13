#!/bin/bash
# round 4: kernel trace + SQ/TA counters of the ragged CRC kernels, round-3
# library against this one, on the few-KiB and 16-64 KiB ragged batches.
#   $1 = output tag; PROF_WL = space-separated workload names below
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4prof}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
V=$PWD/microbench/_variants
declare -A ARGS=(
  [r4100]="--workload ragged --span-min 4100 --span-max 4400 --span-bytes $((4 << 30))"
  [r16k]="--workload ragged --span-min 16384 --span-max 65536 --span-bytes $((4 << 30))"
  [sstc]="--workload sst --sst-types crc32c"
  [blob]="--workload blob"
  [r4096]="--workload ragged --span-min 4096 --span-max 4096 --span-bytes $((4 << 30))"
  [walrec]="--workload walrec"
  [u4300]="--workload crc32c --block-bytes 4300 --blocks 1000000"
  [sstx]="--workload sst --sst-types xxh3"
  [x4k]="--workload xxh3"
  [kv100]="--workload blockkv --kv-value-bytes 100"
  [kv1000]="--workload blockkv --kv-value-bytes 1000"
  [walwrite]="--workload walwrite"
)
PA="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
PB="SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SMEM"
PC="TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE"
for wl in ${PROF_WL:-r4100 r16k}; do
  for v in ${PROF_VARIANTS:-r3base new}; do
    if [ $v = r3base ]; then E="SPEEDB_AMD_AB=1 SPEEDB_AMD_LIB=$V/r3base.so"; else E="-u SPEEDB_AMD_LIB"; fi
    d=$O/${wl}_$v
    mkdir -p $d
    B="python3 bench.py ${ARGS[$wl]} --cpu-seconds 0 --no-verify --steps 5 --warmup 3"
    env $E timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $d/trace -o trace --output-format csv -- $B > $d/bench_trace.txt 2>&1 || { tail -5 $d/bench_trace.txt; exit 1; }
    i=0
    for P in "$PA" "$PB" "$PC"; do
      i=$((i + 1))
      env $E timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace -d $d/pmc$i -o pmc --output-format csv -- $B > $d/bench_pmc$i.txt 2>&1 || { tail -5 $d/bench_pmc$i.txt; exit 1; }
    done
  done
done
python3 - $O <<'PY'
import csv, glob, os, sys, collections
out = sys.argv[1]
for d in sorted(glob.glob(out + "/*_*/")):
    print("==", os.path.basename(d.rstrip("/")))
    for f in glob.glob(d + "trace/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "mck::" in r["Name"]:
                print("  %-60s calls %5s avg_us %8.1f" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for f in glob.glob(d + "pmc*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "mck::" not in k:
                continue
            k = k[:40]
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            n[(k, r["Counter_Name"])] += 1
    for k, dd in acc.items():
        print("  ", k, {c: "%.4g" % (v / n[(k, c)]) for c, v in sorted(dd.items())})
PY

#!/bin/bash
# SQ instruction mix / wait of the block KV kernels (100 B values).
out=gpurun_out/$1
mkdir -p $out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --kernel-trace -d $out/sq -o pmc --output-format csv -- python3 bench.py --workload blockkv --kv-value-bytes ${2:-100} --steps 2 --warmup 1 --settle-ms 0 --no-verify > $out/sq.txt 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD --kernel-trace -d $out/sq2 -o pmc --output-format csv -- python3 bench.py --workload blockkv --kv-value-bytes ${2:-100} --steps 2 --warmup 1 --settle-ms 0 --no-verify > $out/sq2.txt 2>&1 || exit 1
python3 - $out <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for f in glob.glob(out + "/sq*/**/*counter_collection.csv", recursive=True):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "k_block" not in n: continue
        acc[n[:30]][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, d in acc.items():
        print(k, {c: f"{v:.3g}" for c, v in d.items()})
PY

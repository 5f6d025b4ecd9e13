"""Per-kernel mean of every counter in rocprofv3 --pmc CSV output.
   python microbench/pmc_summary.py <dir> <kernel substring> [...]"""
import collections
import csv
import glob
import sys

d, pats = sys.argv[1], sys.argv[2:]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        hit = next((p for p in pats if p in k), None)
        if hit:
            acc[hit][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"  {c:28s} {sum(v) / len(v):.5g}  (n={len(v)})")

#!/usr/bin/env python3
"""Copy one round's GPU-box profile output into the tracked profiles/ tree.

  python profiles/collect.py <tag> [<dest, default tag>]

gpurun_out/bench_<tag>/<wl>.json     -> profiles/<dest>/bench_<wl>.json
gpurun_out/prof_<tag>_<wl>/          -> profiles/<dest>/<wl>/
    trace/trace_kernel_stats.csv, trace/trace_domain_stats.csv (as is)
    trace/trace_kernel_trace.csv     -> trace_mck_kernels.csv (engine kernels only)
    pmc_*/pmc_counter_collection.csv -> pmc_fetch_mck.csv / pmc_write_mck.csv /
                                        pmc_sq_mck.csv (engine kernels only)
    bench_trace.txt                  -> bench_under_rocprof.json
    traffic.json                     -> traffic.json (+ profiles/traffic_<wl>.json)
"""
import csv
import json
import os
import shutil
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(os.path.dirname(HERE), "gpurun_out")


def json_line(path):
    with open(path) as f:
        for ln in f:
            if ln.startswith("{"):
                return ln
    return None


def filter_csv(src, dst, keep_cols=None):
    with open(src) as f, open(dst, "w", newline="") as g:
        r = csv.DictReader(f)
        cols = keep_cols or r.fieldnames
        w = csv.DictWriter(g, fieldnames=cols, extrasaction="ignore")
        w.writeheader()
        for row in r:
            if "mck::" in row.get("Kernel_Name", ""):
                w.writerow(row)


def main():
    tag = sys.argv[1]
    dest = sys.argv[2] if len(sys.argv) > 2 else tag
    dst_root = os.path.join(HERE, dest)
    os.makedirs(dst_root, exist_ok=True)
    bdir = os.path.join(OUT, f"bench_{tag}")
    if os.path.isdir(bdir):
        for fn in sorted(os.listdir(bdir)):
            if fn.endswith(".json"):
                ln = json_line(os.path.join(bdir, fn))
                if ln:
                    with open(os.path.join(dst_root, "bench_" + fn), "w") as f:
                        f.write(ln)
    for d in sorted(os.listdir(OUT)):
        if not d.startswith(f"prof_{tag}_"):
            continue
        wl = d[len(f"prof_{tag}_"):]
        src = os.path.join(OUT, d)
        dst = os.path.join(dst_root, wl)
        os.makedirs(dst, exist_ok=True)
        for fn in ("trace_kernel_stats.csv", "trace_domain_stats.csv"):
            p = os.path.join(src, "trace", fn)
            if os.path.exists(p):
                shutil.copy(p, os.path.join(dst, fn))
        kt = os.path.join(src, "trace", "trace_kernel_trace.csv")
        if os.path.exists(kt):
            filter_csv(kt, os.path.join(dst, "trace_mck_kernels.csv"),
                       ["Dispatch_Id", "Kernel_Name", "Grid_Size", "Workgroup_Size", "LDS_Block_Size",
                        "VGPR_Count", "SGPR_Count", "Start_Timestamp", "End_Timestamp"])
        for kind in ("fetch", "write", "sq"):
            p = os.path.join(src, f"pmc_{kind}", "pmc_counter_collection.csv")
            if os.path.exists(p):
                filter_csv(p, os.path.join(dst, f"pmc_{kind}_mck.csv"))
        ln = json_line(os.path.join(src, "bench_trace.txt"))
        if ln:
            with open(os.path.join(dst, "bench_under_rocprof.json"), "w") as f:
                f.write(ln)
        t = os.path.join(src, "traffic.json")
        if os.path.exists(t):
            with open(t) as f:
                tr = json.load(f)
            tr["source"] = f"profiles/{dest}/{wl} (rocprofv3 run of profiles/run_profile.sh {tag} {wl})"
            for p in (os.path.join(dst, "traffic.json"), os.path.join(HERE, f"traffic_{wl}.json")):
                with open(p, "w") as f:
                    json.dump(tr, f, indent=1)
                    f.write("\n")
        print("collected", wl)


if __name__ == "__main__":
    main()

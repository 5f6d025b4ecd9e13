#!/usr/bin/env python3
"""Turn a run_profile.sh output directory into the per-launch HBM traffic
figure bench.py reports as roofline.traffic.

  python profiles/pmc_to_traffic.py gpurun_out/prof_<tag> <workload> [<shape name>]

Reads the bench JSON line of the trace pass (kernel names + config), the
kernel-trace stats (average duration of those kernels), and the FETCH_SIZE /
WRITE_SIZE passes.  Corrections per MI355X_MICROARCH.md (HBM/rocprofv3):
FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts half the
bytes of a 16-B/lane streaming read, so it is doubled; WRITE_SIZE is exact.
Writes profiles/traffic_<workload>.json and prints a summary.
"""
import csv
import json
import os
import re
import sys


def bench_line(path):
    with open(path) as f:
        for ln in f:
            if ln.startswith("{"):
                return json.loads(ln)
    raise SystemExit(f"no bench JSON line in {path}")


def per_launch(path, names, counter):
    vals = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] == counter and any(n in r["Kernel_Name"] for n in names):
                vals.append(float(r["Counter_Value"]))
    return vals


def main():
    d, workload = sys.argv[1], sys.argv[2]
    line = bench_line(os.path.join(d, "bench_trace.txt"))
    kernel = line["roofline"]["kernel"]
    # "(overlapped step)": the bench times a whole step whose kernels run
    # concurrently in pieces (the device WAL writer); traffic is then per
    # step = per-launch average x launches per step
    # "(N launch(es) per step, timed as the step)": one kernel launched N
    # times per step (the one-pass WAL writer), likewise per step
    overlapped = kernel.endswith("(overlapped step)") or kernel.endswith("timed as the step)")
    names = [k.strip() for k in re.sub(r" \([^()]*(\([^()]*\)[^()]*)*\)$", "", kernel).split(" + ")]
    cfg = {k: v for k, v in line["config"].items() if k not in ("workload", "parallelism")}
    stats = {}
    with open(os.path.join(d, "trace", "trace_kernel_stats.csv")) as f:
        for r in csv.DictReader(f):
            stats[r["Name"]] = r
    avg_ns, calls = 0.0, 0
    for name, r in stats.items():
        if any(n in name for n in names):
            avg_ns += float(r["TotalDurationNs"])
            calls += int(r["Calls"])
    # the bench's timed window = the last steps x launches dispatches of the
    # dominant kernel(s) (the warmup launches come first)
    timed_ns = None
    kt = os.path.join(d, "trace", "trace_kernel_trace.csv")
    if os.path.exists(kt):
        with open(kt) as f:
            durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(f)
                    if any(n in r["Kernel_Name"] for n in names)]
        k = line["steps"] * len(names)
        if len(durs) >= k:
            timed_ns = sum(durs[-k:]) / k
    fetch = per_launch(os.path.join(d, "pmc_fetch", "pmc_counter_collection.csv"), names, "FETCH_SIZE")
    write = per_launch(os.path.join(d, "pmc_write", "pmc_counter_collection.csv"), names, "WRITE_SIZE")
    if not fetch or not write:
        raise SystemExit("no counter rows for " + kernel)
    rd = 2 * 1024 * sum(fetch) / len(fetch)
    wr = 1024 * sum(write) / len(write)
    whole_step = "(whole step" in kernel
    if whole_step:
        # alg bytes per STEP of several kernels (blockkv: layout, scans,
        # protect, long-value sweep): every dispatch of the step's kernels,
        # summed, over the steps the run made (= dispatches of the first
        # kernel, launched once per step)
        steps_f = len(per_launch(os.path.join(d, "pmc_fetch", "pmc_counter_collection.csv"), names[:1], "FETCH_SIZE"))
        steps_w = len(per_launch(os.path.join(d, "pmc_write", "pmc_counter_collection.csv"), names[:1], "WRITE_SIZE"))
        rd = 2 * 1024 * sum(fetch) / max(steps_f, 1)
        wr = 1024 * sum(write) / max(steps_w, 1)
        timed_ns = None
    if overlapped:
        m = re.search(r"\((\d+) launch\(es\) per step", kernel)
        # launches per step: stated in the label, else the dispatch count over
        # the warmup + timed steps (an overlapped run without a settle phase)
        per_step = int(m.group(1)) if m else calls / (line["warmup"] + line["steps"])
        rd, wr = rd * per_step, wr * per_step
        timed_ns = None
    alg = line["roofline"]["alg_bytes_per_launch"]
    # a step of passes over a resident image whose last pass is partial (the
    # WAL replay: 10M blocks = 4 x 2,097,152 + 1,611,392): the counters
    # average the actual dispatches, alg_bytes_per_launch is a full pass --
    # compare like with like, and report the traffic per full pass
    c = line["config"]
    scale = 1.0
    if all(k in c for k in ("blocks_per_gpu", "passes", "resident_blocks")):
        scale = c["blocks_per_gpu"] / (c["passes"] * c["resident_blocks"])
    rd, wr = rd / scale, wr / scale
    out = {
        "workload": workload, "kernel": kernel, "config": cfg,
        "hbm_bytes_per_launch": int(rd + wr),
        "read_bytes_per_launch": int(rd), "write_bytes_per_launch": int(wr),
        "alg_bytes_per_launch": alg, "traffic_over_alg": round((rd + wr) / alg, 4),
        "dispatch_scale": round(scale, 6),
        "rocprof_avg_kernel_ns": round(avg_ns / max(calls, 1), 1), "rocprof_calls": calls,
        "rocprof_timed_window_avg_kernel_ns": None if timed_ns is None else round(timed_ns, 1),
        "bench_kernel_avg_ms": line["roofline"]["kernel_avg_ms"],
        "source": os.path.relpath(d),
        "method": "FETCH_SIZE(KiB)*1024*2 (gfx950 16B/lane read correction) + WRITE_SIZE(KiB)*1024, "
                  + ("summed over every kernel of a step, per step" if whole_step else
                     "averaged over the dominant kernel's dispatches")
                  + "; separate --pmc passes with --kernel-trace only"
                  + ("; per full resident pass (dispatch_scale = mean dispatch / full pass)" if scale != 1.0 else ""),
    }
    # (argv[3]: the file's shape name when a workload has several profiled
    # shapes -- bench.py matches a file by workload, config and kernel)
    name = sys.argv[3] if len(sys.argv) > 3 else workload
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), f"traffic_{name}.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")
    print(json.dumps(out))


if __name__ == "__main__":
    main()

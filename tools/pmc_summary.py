#!/usr/bin/env python3
"""Summarise a tools/profile_round.sh output directory into profiles/.

Writes:
  profiles/<tag>_kernel_stats.csv   rocprofv3 --stats summary (kernel durations)
  profiles/<tag>_pmc.json           per-launch PMC values of the dominant kernel
  profiles/pmc_summary.json         what bench.py reads for roofline.traffic
  profiles/<tag>_bench.json         the bench line of the same session

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch (rocprofv3 derived counters,
summed over XCDs).  Per MI355X_MICROARCH.md §HBM, FETCH_SIZE counts 64 B per
TCC_EA0_RDREQ; it under-reports wide coalesced 128-B streaming reads by 2x and
is uncalibrated for other widths.  This kernel's HBM reads are a mix of
streamed batch data (16-B loads) and random 48/64-B record reads, so we
report the raw counter sum (no 2x correction) and state that beside it.
"""
import csv
import json
import os
import shutil
import statistics
import sys

DOMINANT = "k_receive_fast"


def per_dispatch(path, counter):
    vals = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if DOMINANT not in r["Kernel_Name"] or r["Counter_Name"] != counter:
                continue
            vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return list(vals.values())


def main():
    src, tag = sys.argv[1], sys.argv[2]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prof = os.path.join(root, "profiles")
    os.makedirs(prof, exist_ok=True)
    shutil.copy(os.path.join(src, "stats", "run_kernel_stats.csv"),
                os.path.join(prof, f"{tag}_kernel_stats.csv"))
    bench = json.loads(open(os.path.join(src, "bench.json")).read())
    with open(os.path.join(prof, f"{tag}_bench.json"), "w") as f:
        json.dump(bench, f, indent=1)
    fetch = per_dispatch(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = per_dispatch(os.path.join(src, "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE")
    hit = per_dispatch(os.path.join(src, "pmc_l2", "run_counter_collection.csv"), "TCC_HIT_sum")
    miss = per_dispatch(os.path.join(src, "pmc_l2", "run_counter_collection.csv"), "TCC_MISS_sum")
    f_kib, w_kib = statistics.mean(fetch), statistics.mean(write)
    hbm = (f_kib + w_kib) * 1024
    stats = {}
    with open(os.path.join(src, "stats", "run_kernel_stats.csv")) as f:
        for r in csv.DictReader(f):
            if DOMINANT in r["Name"]:
                stats = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6,
                         "min_ms": float(r["MinNs"]) / 1e6, "max_ms": float(r["MaxNs"]) / 1e6}
    pmc = {"kernel": DOMINANT, "workload": bench["config"]["workload"],
           "fetch_kib_per_launch": f_kib, "write_kib_per_launch": w_kib,
           "hbm_bytes_per_launch": hbm,
           "l2_hit_rate": statistics.mean(hit) / (statistics.mean(hit) + statistics.mean(miss)),
           "tcc_hit_per_launch": statistics.mean(hit), "tcc_miss_per_launch": statistics.mean(miss),
           "rocprof_kernel_stats": stats,
           "bench_kernel_ms": bench["roofline"]["kernel_ms"],
           "algorithmic_bytes_per_launch": bench["roofline"]["algorithmic_bytes_per_launch"],
           "note": "FETCH_SIZE+WRITE_SIZE in KiB x 1024, summed over XCDs; no gfx950 2x "
                   "correction applied (random 48/64-B record reads are uncalibrated, "
                   "MI355X_MICROARCH.md §HBM)"}
    with open(os.path.join(prof, f"{tag}_pmc.json"), "w") as f:
        json.dump(pmc, f, indent=1)
    with open(os.path.join(prof, "pmc_summary.json"), "w") as f:
        json.dump(pmc, f, indent=1)
    print(json.dumps(pmc, indent=1))


if __name__ == "__main__":
    main()

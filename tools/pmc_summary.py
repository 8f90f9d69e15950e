#!/usr/bin/env python3
"""Summarise a tools/profile_round.sh output directory into profiles/.

Writes:
  profiles/<tag>_kernel_stats.csv   rocprofv3 --stats summary (kernel durations)
  profiles/<tag>_pmc.json           per-launch PMC values of the dominant kernel
  profiles/pmc_summary.json         what bench.py reads for roofline.traffic
  profiles/<tag>_bench.json         the bench line of the same session

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch (rocprofv3 derived counters,
summed over XCDs).  Per MI355X_MICROARCH.md §HBM, FETCH_SIZE counts 64 B per
TCC_EA0_RDREQ and so under-reports 128-B requests by 2x.  Rather than apply a
blanket correction, the read bytes are taken from the size-bucketed request
counters (TCC_EA0_RDREQ_32B/_64B/_128B, one pass of their own):
  read bytes = 32*RDREQ_32B + 64*RDREQ_64B + 128*RDREQ_128B.
On this kernel every read request is 128 B (streamed batch data and the
random slot-record lines alike), i.e. exactly 2x FETCH_SIZE.  Writes are
WRITE_SIZE (the fast kernel writes only through atomics; the atomic count is
reported beside it).

The fast path launches the dominant kernel once per chunk of a batch
(bench.json: roofline.launches_per_step), so every figure is per step: the
sum over all dispatches divided by the number of steps they make up.
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


def per_step(vals, lps):
    """Sum of the dispatches of one step (the list holds whole steps only)."""
    return statistics.mean(vals) * lps if vals else None


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
    rd = {k: per_dispatch(os.path.join(src, "pmc_rdsize", "run_counter_collection.csv"), c)
          for k, c in ((32, "TCC_EA0_RDREQ_32B_sum"), (64, "TCC_EA0_RDREQ_64B_sum"),
                       (128, "TCC_EA0_RDREQ_128B_sum"))}
    lps = bench["roofline"].get("launches_per_step", 1)
    rd_bytes = sum(k * per_step(v, lps) for k, v in rd.items() if v)
    atom = per_dispatch(os.path.join(src, "pmc_wr", "run_counter_collection.csv"), "TCC_ATOMIC_sum")
    wrreq = per_dispatch(os.path.join(src, "pmc_wr", "run_counter_collection.csv"), "TCC_EA0_WRREQ_sum")
    hit = per_dispatch(os.path.join(src, "pmc_l2", "run_counter_collection.csv"), "TCC_HIT_sum")
    miss = per_dispatch(os.path.join(src, "pmc_l2", "run_counter_collection.csv"), "TCC_MISS_sum")
    f_kib, w_kib = per_step(fetch, lps), per_step(write, lps)
    hbm = rd_bytes + w_kib * 1024
    stats = {}
    with open(os.path.join(src, "stats", "run_kernel_stats.csv")) as f:
        for r in csv.DictReader(f):
            if DOMINANT in r["Name"]:
                stats = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6,
                         "min_ms": float(r["MinNs"]) / 1e6, "max_ms": float(r["MaxNs"]) / 1e6}
    h_s, m_s = per_step(hit, lps), per_step(miss, lps)
    pmc = {"kernel": DOMINANT, "workload": bench["config"]["workload"],
           "launches_per_step": lps,
           "fetch_kib_per_step": f_kib, "write_kib_per_step": w_kib,
           "read_bytes_per_step": rd_bytes,
           "rdreq_by_size_per_step": {str(k): (per_step(v, lps) or 0.0) for k, v in rd.items()},
           "atomics_per_step": per_step(atom, lps),
           "ea_wrreq_per_step": per_step(wrreq, lps),
           "hbm_bytes_per_step": hbm,
           "l2_hit_rate": h_s / (h_s + m_s),
           "tcc_hit_per_step": h_s, "tcc_miss_per_step": m_s,
           "rocprof_kernel_stats": stats,
           "rocprof_kernel_ms_per_step": stats.get("avg_ms", float("nan")) * lps,
           "bench_kernel_ms_per_step": bench["roofline"]["kernel_ms_per_step"],
           "algorithmic_bytes_per_step": bench["roofline"]["algorithmic_bytes_per_step"],
           "note": "per step = sum over the step's launches of the kernel; hbm_bytes = "
                   "size-bucketed EA read requests (32/64/128 B) + WRITE_SIZE; summed over XCDs "
                   "(MI355X_MICROARCH.md §HBM: FETCH_SIZE tallies 64 B per request, so it reads "
                   "half of the 128-B requests this kernel makes)"}
    with open(os.path.join(prof, f"{tag}_pmc.json"), "w") as f:
        json.dump(pmc, f, indent=1)
    with open(os.path.join(prof, "pmc_summary.json"), "w") as f:
        json.dump(pmc, f, indent=1)
    print(json.dumps(pmc, indent=1))


if __name__ == "__main__":
    main()

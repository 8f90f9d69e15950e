#!/usr/bin/env python3
"""Per-kernel, per-step HBM traffic of a tools/profile_workload.sh run.

    python3 tools/pmc_kernels.py gpurun_out/TAG profiles/TAG_kernels.json

Reads (MI355X_MICROARCH.md §HBM): read bytes from the size-bucketed memory
request counters, 32*RDREQ_32B + 64*RDREQ_64B + 128*RDREQ_128B (FETCH_SIZE
tallies 128-B requests at 64 B on gfx950); write bytes from WRITE_SIZE (KiB).
Per step = (sum over the S=3 run - sum over the S=1 run) / 2 per kernel name,
which cancels the setup kernels both runs share.  Kernel durations (average
and per-step total) come from the --stats run's kernel trace: its last three
steps' worth of dispatches.
"""
import csv
import json
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(?:phip::|rocprim::detail::)?([A-Za-z_][A-Za-z0-9_]*)(?:<|\()", name)
    base = m.group(1) if m else name[:60]
    return ("rocprim:" + base) if "rocprim" in name else base


def sums(path, counters):
    out = defaultdict(float)
    with open(path) as f:
        for r in csv.DictReader(f):
            c = r["Counter_Name"]
            if c in counters:
                out[short(r["Kernel_Name"])] += float(r["Counter_Value"]) * counters[c]
    return out


def main():
    src, dst = sys.argv[1], sys.argv[2]
    rdc = {"TCC_EA0_RDREQ_32B_sum": 32, "TCC_EA0_RDREQ_64B_sum": 64, "TCC_EA0_RDREQ_128B_sum": 128}
    rd = [sums(f"{src}/rd{s}/run_counter_collection.csv", rdc) for s in (1, 3)]
    wr = [sums(f"{src}/wr{s}/run_counter_collection.csv", {"WRITE_SIZE": 1024}) for s in (1, 3)]
    names = sorted(set(rd[1]) | set(wr[1]))
    per = {}
    for k in names:
        r = (rd[1].get(k, 0) - rd[0].get(k, 0)) / 2
        w = (wr[1].get(k, 0) - wr[0].get(k, 0)) / 2
        if r > 1e5 or w > 1e5:
            per[k] = {"read_bytes": r, "write_bytes": w}
    dur = defaultdict(list)
    with open(f"{src}/stats/run_kernel_trace.csv") as f:
        for r in csv.DictReader(f):
            dur[short(r["Kernel_Name"])].append(
                (int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    for k, v in per.items():
        d = sorted(dur.get(k, []))
        if d:
            v["avg_ms"] = sum(x[1] for x in d) / len(d) / 1e6
            v["dispatches"] = len(d)
    tot_r = sum(v["read_bytes"] for v in per.values())
    tot_w = sum(v["write_bytes"] for v in per.values())
    out = {"source": src, "per_step_total_read_bytes": tot_r, "per_step_total_write_bytes": tot_w,
           "kernels": dict(sorted(per.items(), key=lambda kv: -(kv[1]["read_bytes"] +
                                                                 kv[1]["write_bytes"])))}
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    for k, v in out["kernels"].items():
        print(f"{k:40s} rd {v['read_bytes']/1e9:8.3f} GB  wr {v['write_bytes']/1e9:8.3f} GB  "
              f"avg {v.get('avg_ms', float('nan')):8.3f} ms x{v.get('dispatches', 0)}")
    print(f"total per step: rd {tot_r/1e9:.3f} GB wr {tot_w/1e9:.3f} GB")


if __name__ == "__main__":
    main()

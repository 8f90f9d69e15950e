#!/usr/bin/env python3
"""Print the mean per-dispatch value of every counter found under a
tools/pmc_passes.sh output directory (all passes), for kernels matching a
substring.  Usage: tools/pmc_read.py gpurun_out/TAG [kernel-substring]"""
import csv
import glob
import os
import statistics
import sys


def main():
    root = sys.argv[1]
    kern = sys.argv[2] if len(sys.argv) > 2 else "k_receive_fast"
    acc = {}
    for path in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
        per = {}
        with open(path) as f:
            for r in csv.DictReader(f):
                if kern not in r["Kernel_Name"]:
                    continue
                key = (r["Counter_Name"], r["Dispatch_Id"])
                per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
        for (c, _), v in per.items():
            acc.setdefault(c, []).append(v)
    for c in sorted(acc):
        v = acc[c]
        print("%-40s n=%-3d mean=%.4g" % (c, len(v), statistics.mean(v)))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""profiles/ from tools/profile_workload.sh runs, one per bench workload.

    python3 tools/pmc_workloads.py ROUND c2=gpurun_out/r02q_c2 c3=... c4=... c5=...

For every workload key:
  profiles/<ROUND>_<key>_kernel_stats.csv  rocprofv3 --stats summary of the run
  profiles/<ROUND>_<key>_kernels.json      per-kernel HBM bytes per step
                                           (tools/pmc_kernels.py's method)
  profiles/<ROUND>_<key>_bench.json        the bench line of the --stats run
and one entry per key in profiles/pmc_summary.json, which bench.py reads for
roofline.traffic: the HBM bytes per step of the bench's dominant kernel (the
sum of the named kernels for C5's two, the product kernels of the whole step
for C3, whose roofline is priced on the step).

Bytes (MI355X_MICROARCH.md §HBM): reads = 32/64/128 x TCC_EA0_RDREQ_{32,64,128}B
(FETCH_SIZE tallies a 128-B request as 64 B on gfx950), writes = WRITE_SIZE
KiB; per step = (S=3 run - S=1 run) / 2, which cancels setup kernels.
"""
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# torch kernels of the bench's own input generation (outside the timed step)
NOT_PRODUCT = ("elementwise", "distribution", "searchsorted", "rocclr", "indexFunc",
               "index_", "reduce_kernel", "fill")


def bench_line(path):
    with open(path) as f:
        for line in f:
            if line.startswith('{"metric"'):
                return json.loads(line)
    raise SystemExit(f"no bench line in {path}")


def main():
    rnd = sys.argv[1]
    prof = os.path.join(ROOT, "profiles")
    summ_path = os.path.join(prof, "pmc_summary.json")
    try:
        summary = json.load(open(summ_path))
        if "kernel" in summary:          # the round-1 single-workload form
            summary = {"c2": summary}
    except (OSError, ValueError):
        summary = {}
    for spec in sys.argv[2:]:
        key, src = spec.split("=", 1)
        out_k = os.path.join(prof, f"{rnd}_{key}_kernels.json")
        subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_kernels.py"), src, out_k],
                       check=True, stdout=subprocess.DEVNULL)
        shutil.copy(os.path.join(src, "stats", "run_kernel_stats.csv"),
                    os.path.join(prof, f"{rnd}_{key}_kernel_stats.csv"))
        bench = bench_line(os.path.join(src, "stats.log"))
        with open(os.path.join(prof, f"{rnd}_{key}_bench.json"), "w") as f:
            json.dump(bench, f, indent=1)
        kern = json.load(open(out_k))["kernels"]
        dom = bench["roofline"]["kernel"]
        if dom == "whole step":
            names = [k for k in kern if not any(s in k for s in NOT_PRODUCT)]
        else:
            names = dom.split("+")
        rd = sum(kern[k]["read_bytes"] for k in names if k in kern)
        wr = sum(kern[k]["write_bytes"] for k in names if k in kern)
        summary[key] = {
            "kernel": dom,
            "kernels_counted": names,
            "workload": bench["config"]["workload"],
            "read_bytes_per_step": rd,
            "write_bytes_per_step": wr,
            "hbm_bytes_per_step": rd + wr,
            "algorithmic_bytes_per_step": bench["roofline"].get("algorithmic_bytes_per_step"),
            "bench_kernel_ms_per_step": bench["roofline"].get("kernel_ms_per_step"),
            # phip_build_id of the library the counters ran on: bench.py uses
            # this entry only for a run of the same build
            "build_id": bench.get("build_id"),
            "source": f"profiles/{rnd}_{key}_kernels.json",
            "note": "per step; reads = size-bucketed TCC_EA0_RDREQ x 32/64/128 B, writes = "
                    "WRITE_SIZE; (S=3 - S=1)/2 over tools/profile_workload.sh runs",
        }
        print(f"{key}: {dom}: rd {rd/1e9:.3f} GB wr {wr/1e9:.3f} GB per step "
              f"(algorithmic {summary[key]['algorithmic_bytes_per_step']/1e9:.3f} GB)")
    with open(summ_path, "w") as f:
        json.dump(summary, f, indent=1)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Print the key figures of bench.py JSON lines: show_bench.py FILE..."""
import json
import sys

for path in sys.argv[1:]:
    for line in open(path):
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        r = d.get("roofline", {})
        print(f"{path}: {d['value'] / 1e9:.3f} G {d['unit']} n_gpus={d['n_gpus']} "
              f"{d['ms_per_step']:.3f} ms/step; {r.get('kernel')} {r.get('kernel_ms_per_step', 0):.3f} ms "
              f"frac {r.get('frac', 0):.3f}")
        print("   ", d["config"]["workload"])
        print("   ", {k: round(v, 3) for k, v in d.get("kernels_ms", {}).items()})
        cb = d.get("cpu_baseline")
        if cb:
            print("    cpu:", {k: v for k, v in cb.items() if k != "sample"})
        o = d.get("owner_routed")
        if o:
            print(f"    owner_routed: {o['value'] / 1e9:.3f} G/s {o['ms_per_step']:.3f} ms/step, "
                  f"merged/step {o['merged_per_step_total']:.0f}")
        extra = {k: v for k, v in d["config"].items() if k in (
            "messages_merged_per_step_rank0", "converged", "buckets_owned_rank0",
            "buckets_created_per_step")}
        if extra:
            print("   ", extra)

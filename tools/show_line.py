"""One-screen summary of a bench.py JSON line: the headline, its kernels and
each object's step, rate, roofline fraction and `verified`."""
import json
import sys

d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric"')][-1])
r = d.get("roofline") or {}
print(f"C2 {d['value'] / 1e9:.2f} G  {d['ms_per_step']:.3f} ms  frac {r.get('frac')}  "
      f"traffic {r.get('traffic')}  build {d.get('build_id')}")
print("  kernels", {k: round(v, 3) for k, v in (d.get("kernels_ms") or {}).items()})
for key in ("c3", "c4", "anti_entropy"):
    o = d.get(key)
    if not isinstance(o, dict):
        continue
    ro = o.get("roofline") or {}
    print(f"{key}: {o.get('value', 0) / 1e9:.2f} G {o.get('unit')}  {o.get('ms_per_step', 0):.3f} ms  "
          f"frac {ro.get('frac')}  verified {o.get('verified')}")
for k, v in (d.get("c2_variants") or {}).items():
    if isinstance(v, dict):
        ro = v["roofline"]
        print(f"variant {k}: {v['value'] / 1e9:.2f} G  {v['ms_per_step']:.3f} ms  kernel "
              f"{ro['kernel_ms_per_step']:.3f} ms  step_frac {ro.get('step_frac', 0):.3f}  "
              f"ordered {v.get('ordered_messages')}  verified {v['verified']}")
cb = d.get("cpu_baseline") or {}
print("cpu_baseline", {k: cb.get(k) for k in ("value", "unit", "cores", "kind")})

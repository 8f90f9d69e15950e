"""Per-dispatch fabric read requests of tools/ubench_req (req_pmc.sh): for
each allocation mode and variant, the 32/64/128-byte TCC_EA0_RDREQ counts
per record read and the bytes they fetch per record, beside the variant's
time (HIP events, time<mode>.log)."""
import csv
import glob
import os
import sys

out = sys.argv[1]
N = 100_000_000
for m in (0, 1, 2):
    times = []
    try:
        with open(os.path.join(out, f"time{m}.log")) as f:
            for line in f:
                if line.startswith("alloc"):
                    parts = line.split()
                    times.append((" ".join(parts[2:-5]), float(parts[-5])))
    except OSError:
        continue
    rows = []
    for p in glob.glob(os.path.join(out, f"pmc{m}", "**", "*counter_collection.csv"), recursive=True):
        with open(p) as f:
            rows += list(csv.DictReader(f))
    disp = {}
    for r in rows:
        name = r.get("Kernel_Name", "")
        if "rec48" not in name and "narrow" not in name:
            continue
        d = int(r.get("Dispatch_Id", 0))
        disp.setdefault(d, {})[r["Counter_Name"]] = float(r["Counter_Value"])
    ds = sorted(disp)
    print(f"alloc mode {m} ({['hipMalloc', 'uncached', 'fine-grained'][m]})")
    print(f"  {'variant':<20} {'ms':>7} {'32B/rec':>8} {'64B/rec':>8} {'128B/rec':>9} {'bytes/rec':>9}")
    for (name, ms), d in zip(times, ds):
        c = disp[d]
        r32 = c.get("TCC_EA0_RDREQ_32B_sum", 0) / N
        r64 = c.get("TCC_EA0_RDREQ_64B_sum", 0) / N
        r128 = c.get("TCC_EA0_RDREQ_128B_sum", 0) / N
        print(f"  {name:<20} {ms:7.3f} {r32:8.3f} {r64:8.3f} {r128:9.3f} "
              f"{32 * r32 + 64 * r64 + 128 * r128:9.1f}")

#!/bin/bash
# Same-box A/B of the round-1 tree (tools/var/r1tree, built from commit d89cfc6)
# against the current tree: C2 bench lines alternating, two runs each.
set -u
OUT=gpurun_out/${1:-ab_r1}
mkdir -p "$OUT"
ROOT=$(pwd)
show() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], '%.3f ms/step' % d['ms_per_step'], 'fast %.4f' % d['roofline']['kernel_ms_per_step'], 'frac %.3f' % d['roofline']['frac'])" "$1" "$2" | tee -a "$OUT/summary.txt"; }
for rep in 1 2; do
  (cd tools/var/r1tree && timeout -k 10 240 python3 -u bench.py --no-cpu --steps 10 --warmup 2 > "$ROOT/$OUT/r1.$rep.log" 2>&1) || { tail -5 "$OUT/r1.$rep.log"; exit 1; }
  show "$OUT/r1.$rep.log" r1
  timeout -k 10 240 python3 -u bench.py --no-cpu --no-routed --steps 10 --warmup 2 > "$OUT/cur.$rep.log" 2>&1 || { tail -5 "$OUT/cur.$rep.log"; exit 1; }
  show "$OUT/cur.$rep.log" cur
done

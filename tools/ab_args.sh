#!/bin/bash
# A/B of bench.py argument sets on one build: bash tools/ab_args.sh OUT LIB "args1" "args2" ...
set -u
OUT=gpurun_out/$1; LIB=$2; shift 2
mkdir -p "$OUT"
for rep in 1 2; do
  k=0
  for a in "$@"; do
    k=$((k+1))
    PATROLHIP_LIB=$LIB timeout -k 10 240 python3 -u bench.py --no-cpu --steps 10 --warmup 2 $a > "$OUT/v$k.$rep.log" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "[$a] rc=$rc"; tail -5 "$OUT/v$k.$rep.log"; exit $rc; fi
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], '| %.3f ms/step' % d['ms_per_step'], 'fast %.4f' % d['roofline']['kernel_ms_per_step'], 'frac %.3f' % d['roofline']['frac'])" "$OUT/v$k.$rep.log" "$a" | tee -a "$OUT/summary.txt"
  done
done

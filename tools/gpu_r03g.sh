#!/bin/bash
# A/B: k_receive_fast with the bloom prefilter (early home-slot read) vs base.
set -u
OUT=gpurun_out/r03g
mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in base bloom; do
    PATROLHIP_LIB=tools/var/$v.so timeout -k 10 240 python3 -u bench.py --no-cpu --no-routed --steps 10 --warmup 2 > "$OUT/$v.$rep.log" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "$v rc=$rc"; tail -5 "$OUT/$v.$rep.log"; exit $rc; fi
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], '%.3f ms/step' % d['ms_per_step'], 'fast %.4f' % d['kernels_ms']['k_receive_fast'], 'frac %.3f' % d['roofline']['frac'])" "$OUT/$v.$rep.log" $v | tee -a "$OUT/summary.txt"
  done
done

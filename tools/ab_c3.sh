#!/bin/bash
# A/B of tuning builds on C3 (both clocks), alternating, each run under its own
# time limit.  Usage: bash tools/ab_c3.sh OUT v1 v2 ...
set -u
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
for rep in 1 2; do
  for v in "$@"; do
    for clk in below ahead; do
      PATROLHIP_LIB=tools/var/$v.so timeout -k 10 240 python3 -u bench.py --workload c3 --no-cpu --steps 5 --warmup 2 --c3-clock $clk > "$OUT/$v.$clk.$rep.log" 2>&1
      rc=$?
      if [ $rc -ne 0 ]; then echo "$v $clk rc=$rc"; tail -5 "$OUT/$v.$clk.$rep.log"; exit $rc; fi
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernels_ms']; print(sys.argv[2], sys.argv[3], '%.3f ms/step' % d['ms_per_step'], 'gather %.3f fold_block %.3f outputs %.3f' % (k.get('k_gather_huge',0), k.get('k_fold_block',0), k.get('k_huge_outputs',0)))" "$OUT/$v.$clk.$rep.log" $v $clk | tee -a "$OUT/summary.txt"
    done
  done
done

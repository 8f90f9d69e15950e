#!/bin/bash
# A/B of tuning builds on the GPU box: bench.py C2 (SoA and --wire) per variant,
# alternating, each run under its own time limit.  Usage: bash tools/ab.sh OUT v1 v2 ...
set -u
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
for rep in 1 2; do
  for v in "$@"; do
    for mode in soa wire; do
      extra=""; [ $mode = wire ] && extra="--wire"
      PATROLHIP_LIB=tools/var/$v.so timeout -k 10 240 python3 -u bench.py --no-cpu --no-routed --steps 10 --warmup 2 $extra > "$OUT/$v.$mode.$rep.log" 2>&1
      rc=$?
      if [ $rc -ne 0 ]; then echo "$v $mode rc=$rc"; tail -5 "$OUT/$v.$mode.$rep.log"; exit $rc; fi
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], '%.3f ms/step' % d['ms_per_step'], 'fast %.4f' % d['kernels_ms']['k_receive_fast'], 'frac %.3f' % d['roofline']['frac'])" "$OUT/$v.$mode.$rep.log" $v $mode | tee -a "$OUT/summary.txt"
    done
  done
done

#!/bin/bash
# A/B of tuning builds on C2 with short names and with 32-byte names:
# bash tools/ab_names.sh OUT v1 v2 ...  (tools/var/<v>.so)
set -u
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
for rep in 1 2; do
  for v in "$@"; do
    for nl in 0 32; do
      extra=""; [ $nl -ne 0 ] && extra="--name-len $nl"
      PATROLHIP_LIB=tools/var/$v.so timeout -k 10 240 python3 -u bench.py --no-cpu --no-routed --steps 10 --warmup 2 $extra > "$OUT/$v.n$nl.$rep.log" 2>&1
      rc=$?
      if [ $rc -ne 0 ]; then echo "$v n$nl rc=$rc"; tail -5 "$OUT/$v.n$nl.$rep.log"; exit $rc; fi
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], '%.3f ms/step' % d['ms_per_step'], 'fast %.4f' % d['kernels_ms']['k_receive_fast'], 'frac %.3f' % d['roofline']['frac'])" "$OUT/$v.n$nl.$rep.log" $v n$nl | tee -a "$OUT/summary.txt"
    done
  done
done

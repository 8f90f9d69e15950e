#!/bin/bash
# Same-box A/B: HEAD library vs the C3 commit's (tools/var/c3base.so): C2 and
# C3 steps, alternating, two rounds; then C2 with the cold merges' atomics
# replaced (timing only: plain stores / dropped).
set -u
O=gpurun_out/r03s2i
mkdir -p $O
export TMPDIR=/tmp
one() {  # one TAG LIB WORKLOAD
  PATROLHIP_LIB=$2 timeout -k 10 300 python3 -u bench.py --workload $3 --no-cpu --no-routed --steps 8 > $O/$1.$3.json 2> $O/$1.$3.err || { tail -5 $O/$1.$3.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], round(d['ms_per_step'],3), {k: round(v,3) for k,v in d.get('kernels_ms',{}).items() if k in ('k_receive_fast','k_classify')})" $O/$1.$3.json $1 $3
}
for rep in 1 2; do
  one head$rep "" c2
  one base$rep tools/var/c3base.so c2
  one head$rep "" c3
  one base$rep tools/var/c3base.so c3
done
one coldstore tools/var/coldstore.so c2
one coldnoatom tools/var/coldnoatom.so c2

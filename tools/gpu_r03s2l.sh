#!/bin/bash
# Route pack unroll A/B (count 2 vs 4 chunks a step, scatter 1/2/3), 100M x 8 owners.
set -u
O=gpurun_out/r03s2l
mkdir -p $O
export TMPDIR=/tmp
one() {  # one TAG LIB
  PATROLHIP_LIB=$2 timeout -k 10 300 python3 -u bench.py --workload route --no-cpu --steps 10 --messages 100000000 --route-world 8 > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['kernels_ms'].items()})" $O/$1.json $1
}
for rep in 1 2; do
  one head$rep ""
  one rc4_$rep tools/var/rc4.so
  one rs1_$rep tools/var/rs1.so
  one rs3_$rep tools/var/rs3.so
done

#!/bin/bash
# Fused classification in k_receive_fast + faster hot sample + tagged route
# directory: receive parity (fused test, full-size C2, clean prefix, dirty),
# route parity, C2 A/B (fused / not, pre-classified segments), route times.
set -o pipefail
O=gpurun_out/r03s2g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_fullsize.py -m gpu -k "fused" > $O/tests1.log 2>&1 || { tail -30 $O/tests1.log; exit 1; }
tail -2 $O/tests1.log
true
true
run() {  # run TAG ENV...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --no-cpu --no-routed --steps 10 > $O/c2_$tag.json 2> $O/c2_$tag.err || { tail -20 $O/c2_$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c2_$tag.json')); print('c2 $tag', round(d['value']/1e9,2), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['kernels_ms'].items()})"
}
run fused PHIP_FUSE_CLS=1
run nofuse X=1
run pre1 PHIP_FUSE_CLS=1 PHIP_CLS_PRE=1
run pre3 PHIP_FUSE_CLS=1 PHIP_CLS_PRE=3
run fused2 PHIP_FUSE_CLS=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$(pwd)/$O/c2stats" -o run -- python3 -u bench.py --no-cpu --no-routed --warmup 1 --steps 5 > $O/c2stats.log 2>&1 || { tail -20 $O/c2stats.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$(pwd)/$O/route_100m" -o run -- python3 -u bench.py --workload route --no-cpu --steps 5 --warmup 1 --messages 100000000 --route-world 8 > $O/route.log 2>&1 || { tail -20 $O/route.log; exit 1; }
grep -h "route_count\|route_scatter" $O/route_100m/run_kernel_stats.csv | cut -d, -f1,4 | sed 's/(.*"//'

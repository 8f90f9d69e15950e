#!/bin/bash
# Route pack: names staged in LDS (dword stores), 12 workgroups per CU,
# count at 4 chunks per step: route/group/C4 parity, route kernel times.
set -o pipefail
O=gpurun_out/r03s2f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_shard.py tests/test_group.py tests/test_fullsize.py -m gpu -k "route or group or c4" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for m in 12500000 100000000; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$(pwd)/$O/route_$m" -o run -- python3 -u bench.py --workload route --no-cpu --steps 5 --warmup 1 --messages $m --route-world 8 > $O/route_$m.log 2>&1 || { tail -20 $O/route_$m.log; exit 1; }
grep -h "route_count\|route_scatter" $O/route_$m/run_kernel_stats.csv | cut -d, -f1,4 | sed 's/(.*)//' 
done
timeout -k 10 300 python -u bench.py --workload route --no-cpu --steps 10 --messages 100000000 --route-world 8 > $O/route.json 2> $O/route.err || { tail -20 $O/route.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/route.json')); print('route 100M', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['kernels_ms'].items()})"

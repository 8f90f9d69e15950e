#!/bin/bash
# Full rehearsal after the route count's fused classification: pytest -m gpu,
# smoke, default bench; route 100M kernels; C3 bench; C2 kernel stats.
set -u
O=gpurun_out/r03s2h
mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu_final.sh r03s2h/final || exit $?
python3 -c "import json; d=json.load(open('$O/final/bench.json')); print('c2', round(d['value']/1e9,2), round(d['ms_per_step'],3), d['kernels_ms'], d['roofline']['frac'], d.get('owner_routed',{}).get('value'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$(pwd)/$O/route_100m" -o run -- python3 -u bench.py --workload route --no-cpu --steps 5 --warmup 1 --messages 100000000 --route-world 8 > $O/route.log 2>&1 || { tail -20 $O/route.log; exit 1; }
grep -v "^W\|^E" $O/route.log | tail -1 > $O/route.json
python3 -c "import json; d=json.load(open('$O/route.json')); print('route 100M', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['kernels_ms'].items()})"
timeout -k 10 300 python -u bench.py --workload c3 --no-cpu --steps 8 > $O/c3.json 2> $O/c3.err || { tail -20 $O/c3.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c3.json')); print('c3', round(d['value']/1e9,2), round(d['ms_per_step'],3))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$(pwd)/$O/c2stats" -o run -- python3 -u bench.py --no-cpu --no-routed --warmup 1 --steps 5 > $O/c2stats.log 2>&1 || { tail -20 $O/c2stats.log; exit 1; }

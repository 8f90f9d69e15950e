#!/bin/bash
# Session-2 start of round 3: full rehearsal of the checkpointed tree
# (pytest -m gpu, smoke, default bench) and C2/C3 kernel stats.
set -u
O=gpurun_out/r03s2a
mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu_final.sh r03s2a/final || exit $?
python3 -c "import json; d=json.load(open('$O/final/bench.json')); print('c2', round(d['value']/1e9,2), round(d['ms_per_step'],3), d['kernels_ms'], d['roofline']['frac'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$(pwd)/$O/c2stats" -o run -- python3 -u bench.py --no-cpu --no-routed --warmup 1 --steps 5 > $O/c2stats.log 2>&1 || { tail -20 $O/c2stats.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$(pwd)/$O/c3stats" -o run -- python3 -u bench.py --workload c3 --no-cpu --warmup 1 --steps 3 > $O/c3stats.log 2>&1 || { tail -20 $O/c3stats.log; exit 1; }
tail -1 $O/c3stats.log

#!/bin/bash
# Kernel timeline of the owner-routing pack (12.5M messages, 8 owners).
set -o pipefail
O=gpurun_out/r03f
mkdir -p $O
export TMPDIR=/tmp
ROOT=$(pwd)
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$ROOT/$O/tr" -o run -- python3 -u bench.py --workload route --messages 12500000 --route-world 8 --no-cpu --warmup 1 --steps 3 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
python3 tools/timeline.py "$O/tr" k_route_classify > $O/timeline.txt && cat $O/timeline.txt

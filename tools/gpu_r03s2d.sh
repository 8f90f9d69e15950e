#!/bin/bash
# Route pack kernel times (12.5M and 100M messages, 8 owners) and C2 step.
set -o pipefail
O=gpurun_out/r03s2d
mkdir -p $O
export TMPDIR=/tmp
for m in 12500000 100000000; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$(pwd)/$O/route_$m" -o run -- python3 -u bench.py --workload route --no-cpu --steps 5 --warmup 1 --messages $m --route-world 8 > $O/route_$m.log 2>&1 || { tail -20 $O/route_$m.log; exit 1; }
done

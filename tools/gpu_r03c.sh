#!/bin/bash
# C3 baseline of this round: bench line, then the kernel timeline.
set -o pipefail
O=gpurun_out/r03c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --workload c3 --no-cpu --steps 5 > $O/c3.json 2> $O/c3.err || { tail -20 $O/c3.err; exit 1; }
cat $O/c3.json
PHIP_FOLD_STATS=1 timeout -k 10 300 python -u bench.py --workload c3 --no-cpu --steps 1 --warmup 1 > $O/c3_dbg.json 2> $O/c3_dbg.err || { tail -20 $O/c3_dbg.err; exit 1; }
grep "^fold" $O/c3_dbg.err | tail -8
bash tools/trace_c3.sh r03c/trace

#!/bin/bash
# C3 kernel timeline on the GPU box: rocprofv3 kernel trace (csv) of a short
# C3 run, summarised by tools/timeline.py into gpurun_out/<TAG>/timeline.txt.
set -u
TAG=${1:-c3trace}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$ROOT/$OUT/tr" -o run -- python3 -u bench.py --workload c3 --no-cpu --warmup 1 --steps 2 "$@" > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
python3 tools/timeline.py "$OUT/tr" > "$OUT/timeline.txt" && cat "$OUT/timeline.txt"

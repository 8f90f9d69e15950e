#!/bin/bash
# One GPU-box session: every bench.py workload mode once, each JSON line kept
# as gpurun_out/<TAG>/<mode>.json (copied into profiles/ by hand afterwards).
# Usage (from the repo root on the box): bash tools/bench_workloads.sh TAG
# Each step has its own time limit; the script stops at the first failure.
set -u
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"

step() {  # step NAME SECONDS ARGS...
  local name=$1 secs=$2; shift 2
  echo "[$(date +%T)] $name" | tee -a "$OUT/steps.log"
  timeout -k 10 "$secs" python3 -u bench.py "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a "$OUT/steps.log"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/$name.log"; exit $rc; fi
  tail -1 "$OUT/$name.log" > "$OUT/$name.json"
}

step c1 300 --workload c1
step c2_wire 300 --wire --no-cpu
step c2_insert 300 --insert --no-cpu
step c2_ring 300 --ring --no-cpu
step c3 300 --workload c3
step c4 300 --workload c4 --no-cpu
step c5 300 --workload c5 --no-cpu
echo done | tee -a "$OUT/steps.log"

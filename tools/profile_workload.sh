#!/bin/bash
# Kernel stats and per-kernel HBM traffic of one bench.py workload.
# Usage (repo root, on the GPU box): bash tools/profile_workload.sh TAG [bench args...]
#   stats   rocprofv3 --kernel-trace --stats over a warmup + 3-step run
#   rdS/wrS PMC passes (read-request sizes; WRITE_SIZE) over runs of S = 1 and
#           S = 3 timed steps with no warmup: per-step bytes of every kernel are
#           (sum over the 3-step run - sum over the 1-step run) / 2, so setup
#           kernels (generation, seeding) cancel out (tools/pmc_kernels.py).
# Each step has its own time limit; the script stops at the first failure.
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "[$(date +%T)] $name" | tee -a "$OUT/steps.log"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a "$OUT/steps.log"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/$name.log"; exit $rc; fi
}
B="bench.py --no-cpu --no-routed"
step stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/stats" -o run -- python3 -u $B --warmup 1 --steps 3 "$@"
for S in 1 3; do
  step rd$S 300 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --output-format csv -d "$ROOT/$OUT/rd$S" -o run -- python3 -u $B --warmup 0 --steps $S "$@"
  step wr$S 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$ROOT/$OUT/wr$S" -o run -- python3 -u $B --warmup 0 --steps $S "$@"
done
echo done | tee -a "$OUT/steps.log"

#!/bin/bash
# One GPU-box session: full bench (with CPU baseline), rocprofv3 kernel trace
# + stats, and separate PMC passes for HBM traffic of the dominant kernel.
# Usage (from the repo root on the box): bash tools/profile_round.sh TAG
# Each step has its own time limit; the script stops at the first failure.
set -u
TAG=${1:-r01}
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

step bench 600 python3 -u bench.py
tail -1 "$OUT/bench.log" > "$OUT/bench.json"
step rocprof_stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/stats" -o run -- python3 -u bench.py --no-cpu --steps 3 --warmup 1
# PMC: one block's worth of counters per pass (MI355X_MICROARCH.md: FETCH_SIZE
# uses 3 TCC slots, WRITE_SIZE 2; they cannot share a pass).
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_receive_fast --output-format csv -d "$ROOT/$OUT/pmc_fetch" -o run -- python3 -u bench.py --no-cpu --steps 2 --warmup 1
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_receive_fast --output-format csv -d "$ROOT/$OUT/pmc_write" -o run -- python3 -u bench.py --no-cpu --steps 2 --warmup 1
step pmc_rdsize 300 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --kernel-include-regex k_receive_fast --output-format csv -d "$ROOT/$OUT/pmc_rdsize" -o run -- python3 -u bench.py --no-cpu --steps 2 --warmup 1
step pmc_wr 300 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_ATOMIC_sum --kernel-include-regex k_receive_fast --output-format csv -d "$ROOT/$OUT/pmc_wr" -o run -- python3 -u bench.py --no-cpu --steps 2 --warmup 1
step pmc_l2 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex k_receive_fast --output-format csv -d "$ROOT/$OUT/pmc_l2" -o run -- python3 -u bench.py --no-cpu --steps 2 --warmup 1
echo done | tee -a "$OUT/steps.log"

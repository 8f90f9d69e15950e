#!/bin/bash
# Counter passes over the dominant kernel of one short bench run (one
# rocprofv3 --pmc run per pass: counters are never split across passes).
# Usage (repo root on the GPU box): bash tools/pmc_passes.sh TAG [REGEX] [bench args...]
set -u
TAG=${1:-pmc}; RX=${2:-k_receive_fast}; shift 2 || true
ARGS=${*:---no-cpu --steps 2 --warmup 1}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
if [ -n "${PMC_PASSES:-}" ]; then IFS=';' read -r -a PASSES <<< "$PMC_PASSES"; else PASSES=(
  "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD"
  "SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_VALU_INT64 SQ_THREAD_CYCLES_VALU SQ_CYCLES SQ_ACTIVE_INST_VMEM"
  "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_TCC_READ_REQ_sum"
  "TCC_HIT_sum TCC_MISS_sum TCC_ATOMIC_sum TCC_EA0_RDREQ_sum"
  "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE GRBM_UTCL2_BUSY"
  "TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_TCC_READ_REQ_LATENCY_sum"
); fi
k=0
for P in "${PASSES[@]}"; do
  k=$((k+1))
  echo "[$(date +%T)] pass $k: $P"
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex "$RX" --output-format csv \
    -d "$ROOT/$OUT/p$k" -o run -- python3 -u bench.py $ARGS > "$OUT/p$k.log" 2>&1
  rc=$?
  echo "[$(date +%T)] pass $k rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/p$k.log"; exit $rc; fi
done

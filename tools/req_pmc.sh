#!/bin/bash
# tools/ubench_req under the fabric read-request counters (VERDICT r5 item
# 2): one rocprofv3 --pmc pass per allocation mode (hipMalloc, uncached,
# fine-grained), each under its own time limit; summarised per dispatch by
# tools/req_summary.py into gpurun_out/TAG/req.txt.
#   bash tools/req_pmc.sh TAG
set -u
TAG=${1:-req}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
for m in 0 1 2; do
  echo "[$(date +%T)] mode $m" | tee -a "$OUT/steps.log"
  timeout -k 10 120 ./tools/ubench_req $m > "$OUT/time$m.log" 2>&1 || { echo "timing mode $m failed"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum \
    --output-format csv -d "$ROOT/$OUT/pmc$m" -o run -- ./tools/ubench_req $m > "$OUT/pmc$m.log" 2>&1 \
    || { echo "pmc mode $m failed"; exit 1; }
done
python3 tools/req_summary.py "$OUT" > "$OUT/req.txt" && cat "$OUT/req.txt"

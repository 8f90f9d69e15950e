#!/bin/bash
# C3 A/B: thread folds on stream4 vs the main stream; wave-fold depth 1/4/8.
set -o pipefail
O=gpurun_out/r03d
mkdir -p $O
export TMPDIR=/tmp
run() { # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --workload c3 --no-cpu --steps 8 > $O/$tag.json 2> $O/$tag.err || { tail -20 $O/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/$tag.json')); k=d['kernels_ms']; print('$tag', round(d['ms_per_step'],3), 'ms', {x: round(k.get(x,0),3) for x in ('k_resolve','k_resolve_pack','k_pack_ops','k_fold_wave','k_fold_thread','k_fold_block2','k_huge_outputs2')})"
}
run base_same PHIP_THREAD_SAME=1 PHIP_WAVE_DEPTH=1 PHIP_C3_UNFUSED=1
run thread4 PHIP_WAVE_DEPTH=1 PHIP_C3_UNFUSED=1
run d4 PHIP_WAVE_DEPTH=4 PHIP_C3_UNFUSED=1
run d8 PHIP_WAVE_DEPTH=8 PHIP_C3_UNFUSED=1
run fused_d4 PHIP_WAVE_DEPTH=4
run fused_d8 PHIP_WAVE_DEPTH=8
run base_same2 PHIP_THREAD_SAME=1 PHIP_WAVE_DEPTH=1 PHIP_C3_UNFUSED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "mixed" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log

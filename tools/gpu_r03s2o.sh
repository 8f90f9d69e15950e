#!/bin/bash
# C3 thread-fold split: parity with the split on, same-box A/B; two-rank rehearsal.
set -u
O=gpurun_out/r03s2o
mkdir -p $O
export TMPDIR=/tmp
PHIP_THREAD_SPLIT=50 timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_fullsize.py tests/test_gpu_parity.py -m gpu -k "c3 or hot_buckets or adversarial or mixed_large" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
one() {  # one TAG ENV...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --workload c3 --no-cpu --steps 8 > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],3))" $O/$tag.json $tag
}
for rep in 1 2; do
  one s0_$rep X=1
  one s30_$rep PHIP_THREAD_SPLIT=30
  one s50_$rep PHIP_THREAD_SPLIT=50
  one s70_$rep PHIP_THREAD_SPLIT=70
done
timeout -k 10 400 python3 -u bench.py --gpus 2 --dist-backend gloo --no-cpu --steps 3 --warmup 1 > $O/n2.json 2> $O/n2.err || { tail -20 $O/n2.err; exit 1; }
tail -1 $O/n2.json | cut -c1-300

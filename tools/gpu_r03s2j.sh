#!/bin/bash
# The fused classification as a separate instantiation: receive parity, C2
# same-box A/B vs the C3 commit's library.
set -u
O=gpurun_out/r03s2j
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_fullsize.py tests/test_gpu_parity.py tests/test_ingest.py -m gpu -k "fused or receive or hot or wire or datagram or ring" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
one() {  # one TAG LIB WORKLOAD
  PATROLHIP_LIB=$2 timeout -k 10 300 python3 -u bench.py --workload $3 --no-cpu --no-routed --steps 10 > $O/$1.$3.json 2> $O/$1.$3.err || { tail -5 $O/$1.$3.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], round(d['ms_per_step'],3), {k: round(v,3) for k,v in d.get('kernels_ms',{}).items() if k in ('k_receive_fast','k_classify')})" $O/$1.$3.json $1 $3
}
for rep in 1 2 3; do
  one head$rep "" c2
  one base$rep tools/var/c3base.so c2
done

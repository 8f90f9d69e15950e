#!/bin/bash
# C5 full-size test; owner-routing pack cost at 8 / 2 owners.
set -o pipefail
O=gpurun_out/r03e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  "tests/test_fullsize.py::test_c5_full_size_anti_entropy_vs_go_merge" > $O/c5.log 2>&1 || { tail -30 $O/c5.log; exit 1; }
tail -2 $O/c5.log
for cfg in "100000000 8" "12500000 8" "100000000 2"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --workload route --messages $1 --route-world $2 --no-cpu > $O/route_$1_$2.json 2> $O/route_$1_$2.err || { tail -20 $O/route_$1_$2.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/route_$1_$2.json')); print('$1 $2', round(d['value']/1e9,2), 'G msg/s', round(d['ms_per_step'],3), 'ms', {k: round(v,3) for k,v in d['kernels_ms'].items()}, d['config'].get('messages_sent_after_combine'))"
done

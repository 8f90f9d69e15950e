#!/bin/bash
# Fused one-GPU anti-entropy join: AE parity tests, C5 bench x2.
set -o pipefail
O=gpurun_out/${TAG:-r03j}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_shard.py tests/test_group.py tests/test_fullsize.py -k "ae_join or anti_entropy" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
timeout -k 10 300 python -u bench.py --workload c5 --no-cpu --steps 10 > $O/c5_$r.json 2> $O/c5_$r.err || { tail -20 $O/c5_$r.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c5_$r.json')); print(d['value']/1e9, d['ms_per_step'], d['roofline'], d.get('converged'), d.get('kernels_ms'))"
done

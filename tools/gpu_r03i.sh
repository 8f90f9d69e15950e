#!/bin/bash
# C3 with flagged segmentation: ordered-path parity, bench x2.
set -o pipefail
O=gpurun_out/r03i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "mixed or small or upsert or dirty or prefix" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
timeout -k 10 300 python -u bench.py --workload c3 --no-cpu --steps 8 > $O/c3_$r.json 2> $O/c3_$r.err || { tail -20 $O/c3_$r.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c3_$r.json')); k=d['kernels_ms']; print(round(d['ms_per_step'],3), 'ms', {x: round(v,3) for x,v in k.items()})"
done

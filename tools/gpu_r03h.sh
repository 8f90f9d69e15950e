#!/bin/bash
# C3 after the segmentation change: parity (ordered-path tests, full-size C3), bench x2, trace.
set -o pipefail
O=gpurun_out/r03h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_replication.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
timeout -k 10 300 python -u bench.py --workload c3 --no-cpu --steps 8 > $O/c3_$r.json 2> $O/c3_$r.err || { tail -20 $O/c3_$r.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c3_$r.json')); k=d['kernels_ms']; print(round(d['ms_per_step'],3), 'ms', {x: round(v,3) for x,v in k.items()})"
done
bash tools/trace_c3.sh r03h/trace > /dev/null && sed -n '1,40p' $O/trace/timeline.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 900 --timeout-method thread "tests/test_fullsize.py::test_c3_full_size_vs_oracle" > $O/full.log 2>&1 || { tail -30 $O/full.log; exit 1; }
tail -2 $O/full.log

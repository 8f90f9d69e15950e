#!/bin/bash
# k_pack_ops on stream2 beside resolve + sort: ordered-path parity, C3 bench + trace.
set -o pipefail
O=gpurun_out/r03s2b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_parity.py tests/test_fullsize.py tests/test_replication.py tests/test_batcher.py -m gpu -k "mixed or take or ordered or c3 or clean_prefix or upsert or dirty or batcher or reply" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u bench.py --workload c3 --no-cpu --steps 8 > $O/c3.json 2> $O/c3.err || { tail -20 $O/c3.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c3.json')); print('c3', round(d['value']/1e9,2), round(d['ms_per_step'],3))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$(pwd)/$O/c3stats" -o run -- python3 -u bench.py --workload c3 --no-cpu --warmup 1 --steps 3 > $O/c3stats.log 2>&1 || { tail -20 $O/c3stats.log; exit 1; }

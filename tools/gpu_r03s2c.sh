#!/bin/bash
# C3: custom segmentation (k_seg_*), block-fold issue priority, stream
# priority: ordered-path parity, then same-box A/B of the C3 step, and a trace.
set -o pipefail
O=gpurun_out/r03s2c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_parity.py tests/test_fullsize.py tests/test_replication.py tests/test_batcher.py -m gpu -k "mixed or take or ordered or c3 or clean_prefix or upsert or dirty or batcher or reply or hot" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
run() {  # run TAG ENV...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --workload c3 --no-cpu --steps 8 > $O/c3_$tag.json 2> $O/c3_$tag.err || { tail -20 $O/c3_$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c3_$tag.json')); print('c3 $tag', round(d['ms_per_step'],3))"
}
run base X=1
run rle PHIP_SEG_RLE=1
run noprio PHIP_FOLD_NOPRIO=1
run sprio PHIP_STREAM_PRIO=1
run base2 X=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$(pwd)/$O/c3stats" -o run -- python3 -u bench.py --workload c3 --no-cpu --warmup 1 --steps 3 > $O/c3stats.log 2>&1 || { tail -20 $O/c3stats.log; exit 1; }

#!/bin/bash
# C3 after the k_seg_finish fix and the sort values from k_resolve: parity,
# same-box A/B (pack placement, huge split, segmentation), fold stats, trace;
# then the route pack profile.
set -o pipefail
O=gpurun_out/r03s2e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_parity.py tests/test_fullsize.py tests/test_replication.py tests/test_batcher.py -m gpu -k "mixed or take or ordered or c3 or clean_prefix or upsert or dirty or batcher or reply or hot or seed or grow" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
run() {  # run TAG ENV...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --workload c3 --no-cpu --steps 8 > $O/c3_$tag.json 2> $O/c3_$tag.err || { tail -20 $O/c3_$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c3_$tag.json')); print('c3 $tag', round(d['ms_per_step'],3))"
}
run base X=1
run after PHIP_PACK_AFTER=1
run first8 PHIP_HUGE_FIRST=8
run first16 PHIP_HUGE_FIRST=16
run rle PHIP_SEG_RLE=1
run base2 X=1
PHIP_FOLD_STATS=1 timeout -k 10 300 python -u bench.py --workload c3 --no-cpu --steps 1 --warmup 0 > $O/c3_stats.json 2> $O/c3_foldstats.err || { tail -20 $O/c3_foldstats.err; exit 1; }
grep "fold" $O/c3_foldstats.err | head -8
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$(pwd)/$O/c3stats" -o run -- python3 -u bench.py --workload c3 --no-cpu --warmup 1 --steps 3 > $O/c3stats.log 2>&1 || { tail -20 $O/c3stats.log; exit 1; }
for m in 12500000 100000000; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$(pwd)/$O/route_$m" -o run -- python3 -u bench.py --workload route --no-cpu --steps 5 --warmup 1 --messages $m --route-world 8 > $O/route_$m.log 2>&1 || { tail -20 $O/route_$m.log; exit 1; }
done

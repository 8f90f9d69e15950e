set -u
O=gpurun_out/r02j
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "mixed or hot_bucket or absorbing or snapshot or clock" > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
PHIP_FOLD_STATS=1 timeout -k 10 200 python bench.py --workload c3 --steps 1 --warmup 1 --no-cpu > $O/c3_below_dbg.json 2> $O/c3_below_dbg.err || exit $?
PHIP_FOLD_STATS=1 timeout -k 10 200 python bench.py --workload c3 --c3-clock ahead --steps 1 --warmup 1 --no-cpu > $O/c3_ahead_dbg.json 2> $O/c3_ahead_dbg.err || exit $?
timeout -k 10 200 python bench.py --workload c3 --no-cpu > $O/c3_below.json 2> $O/c3_below.err || exit $?
timeout -k 10 200 python bench.py --workload c3 --c3-clock ahead --no-cpu > $O/c3_ahead.json 2> $O/c3_ahead.err || exit $?

set -u
O=gpurun_out/r02f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -s --timeout 120 --timeout-method thread -k "mixed or hot_bucket or absorbing or snapshot or clock" > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python bench.py --workload c3 > $O/c3_below.json 2> $O/c3_below.err || exit $?
timeout -k 10 200 python bench.py --workload c3 --c3-clock ahead > $O/c3_ahead.json 2> $O/c3_ahead.err || exit $?
echo benches done
timeout -k 10 600 python -u -m pytest tests/test_fullsize.py -x -v -s -k c3 > $O/fullsize.log 2>&1
echo "fullsize rc=$?"

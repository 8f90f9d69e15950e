set -u
O=gpurun_out/${1:-r02t}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_fullsize.py -k "mixed or hot or c3 or fold or take" > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
PHIP_FOLD_STATS=1 timeout -k 10 300 python bench.py --workload c3 --no-cpu --steps 2 --warmup 1 > $O/c3_dbg.json 2> $O/c3_dbg.err || exit 1
timeout -k 10 300 python bench.py --workload c3 --no-cpu > $O/c3.json 2> $O/c3.err; rc=$?; echo "c3 rc=$rc"; exit $rc

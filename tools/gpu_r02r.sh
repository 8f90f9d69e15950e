set -u
O=gpurun_out/r02r
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_group.py tests/test_shard.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --workload c5 --no-cpu > $O/c5.json 2> $O/c5.err; rc=$?; echo "c5 rc=$rc"; exit $rc

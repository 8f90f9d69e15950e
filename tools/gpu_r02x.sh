set -u
O=gpurun_out/${1:-r02x}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_shard.py tests/test_group.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --workload c4 --no-cpu > $O/c4.json 2> $O/c4.err; rc=$?; echo "c4 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu > $O/c2.json 2> $O/c2.err; rc=$?; echo "c2 rc=$rc"; exit $rc

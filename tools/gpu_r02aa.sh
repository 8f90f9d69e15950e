set -u
O=gpurun_out/r02aa
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_group.py tests/test_shard.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --workload c5 --no-cpu > $O/c5.json 2> $O/c5.err || exit 1
timeout -k 10 300 python bench.py --workload c4 --no-cpu > $O/c4.json 2> $O/c4.err || exit 1
PFX=r02r bash tools/gpu_r02q.sh c4 c5

set -u
O=gpurun_out/${1:-s2m}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u bench.py --workload c3 > $O/c3.json 2> $O/c3.err || exit 1
timeout -k 10 300 python3 -u bench.py > $O/c2.json 2> $O/c2.err || exit 1
python3 tools/show_bench.py $O/c3.json $O/c2.json 2>/dev/null || tail -c 600 $O/c3.json

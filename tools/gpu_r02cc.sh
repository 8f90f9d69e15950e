set -u
O=gpurun_out/r02dd
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "name or datagram or receive or hot" > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for L in 15 20 32; do timeout -k 10 300 python bench.py --name-len $L --no-routed --no-cpu > $O/c2_names$L.json 2> $O/c2_names$L.err || exit 1; done
timeout -k 10 300 python bench.py --no-routed --no-cpu > $O/c2.json 2> $O/c2.err || exit 1

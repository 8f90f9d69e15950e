set -u
O=gpurun_out/${1:-r02z}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_batcher.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for th in 1 16 64; do
  timeout -k 10 120 ./tools/take_load $th 2000 20 100000 >> $O/take_load.jsonl 2> $O/take_load.err || exit 1
done
cat $O/take_load.jsonl

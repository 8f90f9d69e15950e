set -u
O=gpurun_out/r02b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_batcher.py -x -v -s --timeout 120 --timeout-method thread > $O/batcher_tests.log 2>&1
rc=$?; echo "batcher tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for T in 1 16 64 256; do
  timeout -k 10 120 ./tools/take_load $T 2000 20 100000 >> $O/take_load.jsonl 2>>$O/take_load.err || exit $?
done
for W in 0 100; do
  timeout -k 10 120 ./tools/take_load 64 2000 $W 100000 >> $O/take_load.jsonl 2>>$O/take_load.err || exit $?
done
echo take_load done
timeout -k 10 200 python bench.py --workload c3 > $O/c3_below.json 2> $O/c3_below.err || exit $?
timeout -k 10 200 python bench.py --workload c3 --c3-clock ahead > $O/c3_ahead.json 2> $O/c3_ahead.err || exit $?
echo benches done
bash tools/profile_workload.sh r02b_c3 --workload c3 || exit $?
bash tools/profile_workload.sh r02b_c3a --workload c3 --c3-clock ahead || exit $?

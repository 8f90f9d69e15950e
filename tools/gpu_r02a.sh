set -u
mkdir -p gpurun_out/r02a
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread > gpurun_out/r02a/tests.log 2>&1
rc=$?
echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 240 python bench.py > gpurun_out/r02a/bench.json 2> gpurun_out/r02a/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python bench.py --gpus 2 --dist-backend gloo --no-cpu --steps 3 --warmup 1 > gpurun_out/r02a/bench_g2.json 2> gpurun_out/r02a/bench_g2.err
echo "bench2 rc=$?"

set -u
O=gpurun_out/r02d
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_group.py tests/test_batcher.py -v -s --timeout 120 --timeout-method thread > $O/tests.log 2>&1
echo "tests rc=$?"

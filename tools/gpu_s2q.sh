set -u
O=gpurun_out/${1:-s2q}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "mixed or hot or c3 or dirty" > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_fullsize.py -k c3 > $O/tests_full.log 2>&1
rc=$?; echo "fullsize rc=$rc"; tail -2 $O/tests_full.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  for v in head outs; do
    PATROLHIP_LIB=tools/var/$v.so timeout -k 10 200 python3 -u bench.py --workload c3 --no-cpu --steps 5 --warmup 1 > $O/c3_$v.$rep.log 2>&1 || { tail -5 $O/c3_$v.$rep.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], '%.3f ms/step' % d['ms_per_step'], {k: round(v,3) for k,v in d['kernels_ms'].items() if 'huge' in k or 'fold' in k})" $O/c3_$v.$rep.log $v | tee -a $O/summary.txt
  done
done

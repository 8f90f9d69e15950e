set -u
O=gpurun_out/${1:-s2s}
mkdir -p $O
PATROLHIP_LIB=tools/var/fillmain.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_ingest.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  for v in head fillmain; do
    PATROLHIP_LIB=tools/var/$v.so timeout -k 10 200 python3 -u bench.py --workload c1 --no-cpu --steps 20 --warmup 3 > $O/c1_$v.$rep.log 2>&1 || { tail -5 $O/c1_$v.$rep.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], '%.4f ms/step' % d['ms_per_step'], {k: round(v,4) for k,v in d['kernels_ms'].items()})" $O/c1_$v.$rep.log $v | tee -a $O/summary.txt
  done
done

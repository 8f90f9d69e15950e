set -u
O=gpurun_out/${1:-s2d}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "mixed or hot or c3" > $O/tests_hot.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests_hot.log; [ $rc -ne 0 ] && exit $rc
run() {  # label env...
  local lab=$1; shift
  env "$@" timeout -k 10 200 python3 -u bench.py --workload c3 --no-cpu --steps 5 --warmup 1 > $O/c3_$lab.$rep.log 2>&1 || { tail -5 $O/c3_$lab.$rep.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], '%.3f ms/step' % d['ms_per_step'], {k: round(v,3) for k,v in d['kernels_ms'].items() if 'huge' in k or 'fold' in k})" $O/c3_$lab.$rep.log $lab | tee -a $O/summary.txt
}
for rep in 1 2; do
  run beside_f0 PHIP_C3_GATHER_BESIDE=1 PHIP_HUGE_FIRST=0
  run first_f0 PHIP_HUGE_FIRST=0
  run first_f4 PHIP_HUGE_FIRST=4
  run beside_f4 PHIP_C3_GATHER_BESIDE=1 PHIP_HUGE_FIRST=4
done

set -u
O=gpurun_out/r02p
mkdir -p $O
echo "[$(date +%T)] tests"
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
run() {  # run NAME SECONDS ARGS...
  local name=$1 secs=$2; shift 2
  echo "[$(date +%T)] $name"
  timeout -k 10 $secs python bench.py "$@" > $O/$name.json 2> $O/$name.err
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $O/$name.err; exit $rc; fi
}
run c2_names32 300 --name-len 32 --no-routed --no-cpu
run c2 300 --no-routed --no-cpu

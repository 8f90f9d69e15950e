set -u
O=gpurun_out/r02m
mkdir -p $O
run() {  # run NAME SECONDS ARGS...
  local name=$1 secs=$2; shift 2
  echo "[$(date +%T)] $name"
  timeout -k 10 $secs python bench.py "$@" > $O/$name.json 2> $O/$name.err
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $O/$name.err; exit $rc; fi
}
run c2 300
run c4 300 --workload c4 --no-cpu
run c5 300 --workload c5 --no-cpu
run c4_125m 400 --workload c4 --keys 125000000 --log2-slots 28 --no-cpu
run c2_names32 300 --name-len 32 --no-routed
run c1 300 --workload c1
run c2_g2gloo 300 --gpus 2 --dist-backend gloo --no-cpu --steps 3 --warmup 1

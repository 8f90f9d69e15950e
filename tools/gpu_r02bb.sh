set -u
O=gpurun_out/r02bb
mkdir -p $O
run() {  # run NAME SECONDS ARGS...
  local name=$1 secs=$2; shift 2
  echo "[$(date +%T)] $name"
  timeout -k 10 $secs python bench.py "$@" > $O/$name.json 2> $O/$name.err
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $O/$name.err; exit $rc; fi
}
run c2 300 --no-routed
run c2_uniform 300 --zipf 0 --no-routed --no-cpu
run c2_names15 300 --name-len 15 --no-routed --no-cpu
run c2_names23 300 --name-len 23 --no-routed --no-cpu
run c2_names40 300 --name-len 40 --no-routed --no-cpu
run c2_wire 300 --wire --no-routed --no-cpu
run c4_125m 400 --workload c4 --keys 125000000 --log2-slots 28 --no-cpu
run c4_uniform 300 --workload c4 --zipf 0 --no-cpu
run c3_ahead 300 --workload c3 --c3-clock ahead --no-cpu
run c2_insert 300 --insert --log2-slots 27 --no-routed --no-cpu

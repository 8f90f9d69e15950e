#!/bin/bash
# One gpurun call as a list of named steps, each under its own time limit;
# the call stops at the first step that fails (no GPU step after a fault,
# abort or time limit).  Every log lands in gpurun_out/TAG/.
#
#   bash tools/gpu.sh TAG 'STEP [ARGS...]' ['STEP [ARGS...]' ...]   ('%' in an ARG = a space)
#
# steps:
#   tests [PYTEST ARGS]   pytest -m gpu (e.g. 'tests -k fullsize')      tests.log
#   smoke                 __graft_entry__.smoke()                        smoke.log
#   bench NAME [ARGS]     python bench.py ARGS                           NAME.json / NAME.err
#   benchv NAME VAR [ARGS] bench.py ARGS on tools/var/VAR.so (tools/build_variants.sh)
#   gloo2 NAME [ARGS]     bench.py --gpus 2 --dist-backend gloo ARGS     (two ranks, one GPU)
#   prof NAME [ARGS]      rocprofv3 --kernel-trace --stats over bench.py NAME/ (+ NAME.json)
#   profpy NAME SCRIPT [ARGS]  rocprofv3 --kernel-trace --stats over python3 SCRIPT ARGS   NAME/
#   passes NAME REGEX [ARGS]  tools/pmc_passes.sh over kernels matching REGEX (PMC_PASSES: ';'-list)
#   pmc NAME [ARGS]       tools/profile_workload.sh TAG/NAME ARGS        (counter passes)
#   py NAME SCRIPT [ARGS] python3 -u SCRIPT ARGS                         NAME.log
#   sh NAME SCRIPT [ARGS] bash SCRIPT ARGS                               NAME.log
set -u
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
ROOT=$(pwd)
run() {  # run SECONDS LOG CMD...
  local secs=$1 log=$2; shift 2
  echo "[$(date +%T)] $*" | tee -a "$O/steps.log"
  timeout -k 10 "$secs" "$@" > "$log" 2>&1
  local rc=$?
  echo "[$(date +%T)] rc=$rc" | tee -a "$O/steps.log"
  if [ $rc -ne 0 ]; then tail -30 "$log"; exit $rc; fi
}
for spec in "$@"; do
  set -- $spec
  kind=$1; shift
  # '%' in an argument stands for a space (e.g. -k 'group%or%route')
  args=()
  for a in "$@"; do args+=("${a//%/ }"); done
  set -- "${args[@]}"
  case $kind in
    tests)
      [ $# -eq 0 ] && set -- tests
      run 1000 "$O/tests.log" python3 -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu "$@"
      tail -3 "$O/tests.log" ;;
    smoke)
      run 300 "$O/smoke.log" python3 -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)
      name=$1; shift
      echo "[$(date +%T)] bench $name: $*" | tee -a "$O/steps.log"
      timeout -k 10 900 python3 -u bench.py "$@" > "$O/$name.json" 2> "$O/$name.err"
      rc=$?; echo "[$(date +%T)] rc=$rc" | tee -a "$O/steps.log"
      tail -1 "$O/$name.json" | cut -c1-600
      if [ $rc -ne 0 ]; then tail -30 "$O/$name.err"; exit $rc; fi ;;
    benchv)   # benchv NAME VARIANT [ARGS]: bench.py on tools/var/VARIANT.so
      name=$1; var=$2; shift 2
      echo "[$(date +%T)] bench $name ($var): $*" | tee -a "$O/steps.log"
      PATROLHIP_LIB=tools/var/$var.so timeout -k 10 900 python3 -u bench.py "$@" > "$O/$name.json" 2> "$O/$name.err"
      rc=$?; echo "[$(date +%T)] rc=$rc" | tee -a "$O/steps.log"
      tail -1 "$O/$name.json" | cut -c1-600
      if [ $rc -ne 0 ]; then tail -30 "$O/$name.err"; exit $rc; fi ;;
    gloo2)
      name=$1; shift
      echo "[$(date +%T)] gloo2 $name: $*" | tee -a "$O/steps.log"
      timeout -k 10 900 python3 -u bench.py --gpus 2 --dist-backend gloo "$@" > "$O/$name.json" 2> "$O/$name.err"
      rc=$?; echo "[$(date +%T)] rc=$rc" | tee -a "$O/steps.log"
      tail -1 "$O/$name.json" | cut -c1-600
      if [ $rc -ne 0 ]; then tail -30 "$O/$name.err"; exit $rc; fi ;;
    prof)
      name=$1; shift
      run 600 "$O/$name.log" rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$O/$name" -o run -- python3 -u bench.py "$@"
      grep '^{"metric"' "$O/$name.log" > "$O/$name.json" || true ;;
    profpy)
      name=$1; shift
      run 600 "$O/$name.log" rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$O/$name" -o run -- python3 -u "$@" ;;
    passes)   # passes NAME REGEX [BENCH ARGS]: tools/pmc_passes.sh counter passes ($PMC_PASSES)
      name=$1; rx=$2; shift 2
      run 1200 "$O/$name.passes.log" bash tools/pmc_passes.sh "$TAG/$name" "$rx" "$@" ;;
    pmc)
      name=$1; shift
      run 1200 "$O/$name.pmc.log" bash tools/profile_workload.sh "$TAG/$name" "$@" ;;
    py)
      name=$1; shift
      run 900 "$O/$name.log" python3 -u "$@"
      tail -5 "$O/$name.log" ;;
    sh)       # sh NAME SCRIPT [ARGS]: bash SCRIPT ARGS (its own steps time-limited)
      name=$1; shift
      run 900 "$O/$name.log" bash "$@"
      tail -15 "$O/$name.log" ;;
    *) echo "unknown step $kind"; exit 2 ;;
  esac
done
echo "all steps done" | tee -a "$O/steps.log"

# Round-2 profiles: kernel stats + per-kernel HBM traffic of the given workloads.
set -u
for w in "$@"; do
  case $w in
    c2) bash tools/profile_workload.sh ${PFX:-r02q}_c2 || exit 1 ;;
    c3) bash tools/profile_workload.sh ${PFX:-r02q}_c3 --workload c3 || exit 1 ;;
    c4) bash tools/profile_workload.sh ${PFX:-r02q}_c4 --workload c4 || exit 1 ;;
    c5) bash tools/profile_workload.sh ${PFX:-r02q}_c5 --workload c5 || exit 1 ;;
  esac
done

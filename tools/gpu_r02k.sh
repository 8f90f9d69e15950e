set -u
O=gpurun_out/r02k
mkdir -p $O
PHIP_FOLD_STATS=1 timeout -k 10 200 python bench.py --workload c3 --steps 1 --warmup 1 --no-cpu > $O/c3_below_dbg.json 2> $O/c3_below_dbg.err || exit $?

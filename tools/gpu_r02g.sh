set -u
O=gpurun_out/r02g
mkdir -p $O
PHIP_FOLD_STATS=1 timeout -k 10 200 python bench.py --workload c3 --steps 1 --warmup 1 --no-cpu > $O/c3_below.json 2> $O/c3_below.err || exit $?
PHIP_FOLD_STATS=1 timeout -k 10 200 python bench.py --workload c3 --c3-clock ahead --steps 1 --warmup 1 --no-cpu > $O/c3_ahead.json 2> $O/c3_ahead.err || exit $?

#!/bin/bash
# End-of-session rehearsal (pytest -m gpu, smoke, bench), then a two-rank
# (gloo) bench on the one GPU.
set -u
O=gpurun_out/r03s2p
mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu_final.sh r03s2p/final || exit $?
python3 -c "import json; d=json.load(open('$O/final/bench.json')); print('c2', round(d['value']/1e9,2), round(d['ms_per_step'],3), d['kernels_ms'], d['roofline']['frac'])"
timeout -k 10 400 python3 -u bench.py --gpus 2 --dist-backend gloo --no-cpu --steps 3 --warmup 1 > $O/n2.json 2> $O/n2.err || { tail -20 $O/n2.err; exit 1; }
tail -1 $O/n2.json | cut -c1-300

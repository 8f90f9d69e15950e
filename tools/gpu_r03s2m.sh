#!/bin/bash
# Round-3 (second session) profiles: rocprofv3 stats + per-kernel HBM bytes
# for C2, C3 and the 100M x 8-owner route pack.
set -u
bash tools/profile_workload.sh r03s2m_c2 || exit $?
bash tools/profile_workload.sh r03s2m_c3 --workload c3 || exit $?
bash tools/profile_workload.sh r03s2m_route --workload route --messages 100000000 --route-world 8 || exit $?
# two ranks on the one GPU (gloo barriers, the torch routing glue): the
# launcher, max-over-ranks timing and the owner-routed leg at world 2
timeout -k 10 400 python3 -u bench.py --gpus 2 --dist-backend gloo --no-cpu --steps 3 --warmup 1 > gpurun_out/r03s2m_n2.json 2> gpurun_out/r03s2m_n2.err || { tail -20 gpurun_out/r03s2m_n2.err; exit 1; }
tail -1 gpurun_out/r03s2m_n2.json | cut -c1-400

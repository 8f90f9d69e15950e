#!/bin/bash
# Route pack without per-owner ballot rounds (LDS atomics in the count,
# packed DPP scans in the scatter): route/group parity, route bench, C5, counters.
set -o pipefail
O=gpurun_out/r03m
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_shard.py tests/test_group.py tests/test_fullsize.py -m gpu -k "route or group or c4 or ae_join or anti_entropy" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for m in 12500000 100000000; do
timeout -k 10 300 python -u bench.py --workload route --no-cpu --steps 10 --messages $m --route-world 8 > $O/route_$m.json 2> $O/route_$m.err || { tail -20 $O/route_$m.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/route_$m.json')); print('route $m', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['kernels_ms'].items()})"
done
timeout -k 10 300 python -u bench.py --workload c5 --no-cpu --steps 10 > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c5.json')); print('c5', round(d['value']/1e9,2), round(d['ms_per_step'],3), d['kernels_ms'])"
timeout -k 10 300 python -u bench.py --no-cpu --steps 10 > $O/c2.json 2> $O/c2.err || { tail -20 $O/c2.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c2.json')); print('c2', round(d['value']/1e9,2), round(d['ms_per_step'],3), d.get('owner_routed',{}).get('value'))"
PMC_PASSES="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD;SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_VALU_INT64 SQ_THREAD_CYCLES_VALU SQ_CYCLES SQ_ACTIVE_INST_VMEM" \
  bash tools/pmc_passes.sh r03m_route 'k_route_count|k_route_scatter' --workload route --no-cpu --steps 2 --warmup 1 --messages 12500000 --route-world 8

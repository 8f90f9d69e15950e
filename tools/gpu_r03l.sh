#!/bin/bash
# k_ae_join: plain vs non-temporal loads (PHIP_AE_NT), C5 bench x2 each.
set -o pipefail
O=gpurun_out/r03l
mkdir -p $O
export TMPDIR=/tmp
for v in 0 1 0 1; do
PHIP_AE_NT=$v timeout -k 10 300 python -u bench.py --workload c5 --no-cpu --steps 10 > $O/c5_$v.json 2> $O/c5_$v.err || { tail -20 $O/c5_$v.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c5_$v.json')); print('NT=$v', round(d['value']/1e9,2), round(d['ms_per_step'],3), d['kernels_ms'])"
done
# route pack counters (12.5M messages, 8 owners: one rank's share of the owner-routed line at 8 GPUs)
PMC_PASSES="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD;SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_VALU_INT64 SQ_THREAD_CYCLES_VALU SQ_CYCLES SQ_ACTIVE_INST_VMEM;TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum;GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM" \
  bash tools/pmc_passes.sh r03l_route 'k_route_count|k_route_scatter' --workload route --no-cpu --steps 2 --warmup 1 --messages 12500000 --route-world 8

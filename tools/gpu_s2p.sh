set -u
O=gpurun_out/${1:-s2p}
mkdir -p $O
for rep in 1 2; do
  for f in 4 8 16; do
    PHIP_HUGE_FIRST=$f timeout -k 10 200 python3 -u bench.py --workload c3 --no-cpu --steps 5 --warmup 1 > $O/c3_f$f.$rep.log 2>&1 || { tail -5 $O/c3_f$f.$rep.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('first', sys.argv[2], '%.3f ms/step' % d['ms_per_step'], {k: round(v,3) for k,v in d['kernels_ms'].items() if 'huge' in k or 'fold' in k})" $O/c3_f$f.$rep.log $f | tee -a $O/summary.txt
  done
done

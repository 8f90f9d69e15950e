set -u
O=gpurun_out/${1:-s2t}
mkdir -p $O
for rep in 1 2 3; do
  for v in side main; do
    env $( [ $v = main ] && echo PHIP_FILL_MAIN=1 || echo X=1 ) timeout -k 10 200 python3 -u bench.py --no-cpu --no-routed --steps 10 --warmup 2 > $O/$v.$rep.log 2>&1 || { tail -5 $O/$v.$rep.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], '%.4f ms/step' % d['ms_per_step'], {k: round(v,4) for k,v in d['kernels_ms'].items()})" $O/$v.$rep.log $v | tee -a $O/summary.txt
  done
done

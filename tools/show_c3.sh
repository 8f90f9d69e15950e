# summarise a C3 GPU run directory: bench lines and fold stats
D=$1
for f in c3_below c3_ahead; do
python3 - "$D/$f.json" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l)
        print(sys.argv[1].split('/')[-1], round(d['value'] / 1e9, 3), 'G ops/s', round(d['ms_per_step'], 3), 'ms')
        print('  ', {k: round(v, 3) for k, v in d['kernels_ms'].items()})
PY
grep "^fold\[" $D/${f}_dbg.err 2>/dev/null | tail -3
done

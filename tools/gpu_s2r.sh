set -u
O=gpurun_out/${1:-s2r}
mkdir -p $O
for w in c1 c4 c5; do
  timeout -k 10 300 python3 -u bench.py --workload $w $( [ $w != c1 ] && echo --no-cpu ) > $O/$w.json 2> $O/$w.err || { tail -5 $O/$w.err; exit 1; }
done
timeout -k 10 300 python3 -u bench.py --workload c4 --no-cpu --keys 125000000 --log2-slots 28 > $O/c4_125m.json 2> $O/c4_125m.err || { tail -5 $O/c4_125m.err; exit 1; }
timeout -k 10 300 python3 -u bench.py --no-cpu --no-routed --name-len 32 > $O/c2_n32.json 2> $O/c2_n32.err || exit 1
timeout -k 10 300 python3 -u bench.py --no-cpu --no-routed --wire > $O/c2_wire.json 2> $O/c2_wire.err || exit 1
python3 tools/show_bench.py $O/*.json

# round 6, final tree with its hash-matched PMC profile (r06y) committed: a bench line per
# configuration, so every line carries the profiled bound (the default line with its CPU baselines,
# config 6 with its reference estimate); smoke once more
export TMPDIR=/tmp
OUT=gpurun_out/r06final3
mkdir -p $OUT
sha256sum topotrafficrl_amd/lib/*.so > $OUT/sha.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1 || exit $?
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
for c in 2 3 5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $OUT/bench_c$c.json 2>> $OUT/bench.err || exit $?
done
timeout -k 10 300 python bench.py --config 4 --dtype f32 --no-cpu-baseline > $OUT/bench_c4_f32.json 2>> $OUT/bench.err || exit $?
timeout -k 10 400 python bench.py --config 6 > $OUT/bench_c6.json 2>> $OUT/bench.err || exit $?
for f in $OUT/bench*.json; do echo $f; python -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d['roofline']; print(round(d['ms_per_step'],4), round(r['kernel_ms'],4), '%.4g'%d['value'], r['bound'], round(r['frac'],3), r.get('traffic'))
"; done

# round 6, final tree (after the progress priorities): the GPU suite (parity log), smoke, the default bench line (config 4 with its CPU
# baselines) and a bench line per configuration (config 6 with its CPU baselines)
export TMPDIR=/tmp
OUT=gpurun_out/r06final2
mkdir -p $OUT
sha256sum topotrafficrl_amd/lib/*.so > $OUT/sha.txt
TTRL_PARITY_LOG=$OUT/parity.json timeout -k 10 600 python -u -m pytest tests -m gpu -q -rs --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/gpu_tests.txt; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1 || exit $?
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
for c in 2 3 5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $OUT/bench_c$c.json 2>> $OUT/bench.err || exit $?
done
timeout -k 10 400 python bench.py --config 6 > $OUT/bench_c6.json 2>> $OUT/bench.err || exit $?
timeout -k 10 300 python bench.py --config 6 --no-cpu-baseline --steps 200 > $OUT/bench_c6_200.json 2>> $OUT/bench.err || exit $?
timeout -k 10 300 python bench.py --config 4 --dtype f32 --no-cpu-baseline > $OUT/bench_c4_f32.json 2>> $OUT/bench.err || exit $?
for f in $OUT/bench*.json; do echo $f; python -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1]); print(round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), '%.4g'%d['value'], d['roofline']['bound'])
"; done

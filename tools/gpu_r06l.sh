# round 6: bench with the per-launch timing events moved out of the timed loop, configs 4, 2, 3, 6
export TMPDIR=/tmp
OUT=gpurun_out/r06l
mkdir -p $OUT
for c in 4 2 3; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline >> $OUT/bench_c$c.json 2>> $OUT/err || exit $?
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline >> $OUT/bench_c$c.json 2>> $OUT/err || exit $?
done
timeout -k 10 300 python bench.py --config 6 --no-cpu-baseline --steps 200 >> $OUT/bench_c6_200.json 2>> $OUT/err || exit $?
for f in $OUT/*.json; do echo $f; python -c "
import json,sys
for l in open('$f'):
    d=json.loads(l); print(round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), '%.4g'%d['value'])
"; done

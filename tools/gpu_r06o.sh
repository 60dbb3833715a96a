# round 6 (r06o): as r06n with the peel only in the 128/256-slot and road-network instances; the meta-action peeled off the frame loop, the ego's speed index written where it
# changes, kin_observe compiled out of the grid instance, the 128-slot SAT queue index laundered
# (config 3's instance 20 -> 0 B/lane of scratch): the whole GPU suite, then configs 4, 2, 3, 6
# against the previous build (tools/_ab/lib_prev.so), alternated on one box
export TMPDIR=/tmp
OUT=gpurun_out/r06o
mkdir -p $OUT
LIB=topotrafficrl_amd/lib/libttrl_mi355x.so
cp $LIB /tmp/lib_new.so || exit 1
TTRL_PARITY_LOG=$OUT/parity.json timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for c in 4 2 3; do
    cp /tmp/lib_new.so $LIB && timeout -k 10 200 python bench.py --config $c --no-cpu-baseline >> $OUT/new_c$c.json 2>> $OUT/err || exit $?
    cp tools/_ab/lib_prev.so $LIB && timeout -k 10 200 python bench.py --config $c --no-cpu-baseline >> $OUT/prev_c$c.json 2>> $OUT/err || exit $?
  done
done
for r in 1 2; do
  cp /tmp/lib_new.so $LIB && timeout -k 10 200 python bench.py --config 6 --no-cpu-baseline --steps 200 >> $OUT/new_c6.json 2>> $OUT/err || exit $?
  cp tools/_ab/lib_prev.so $LIB && timeout -k 10 200 python bench.py --config 6 --no-cpu-baseline --steps 200 >> $OUT/prev_c6.json 2>> $OUT/err || exit $?
done
cp /tmp/lib_new.so $LIB
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o c4 -- python3 bench.py --config 4 --no-cpu-baseline > $OUT/trace_c4.json 2> $OUT/trace_c4.err || exit $?
for f in $OUT/new_c*.json $OUT/prev_c*.json; do echo $f; python -c "
import json
for l in open('$f'):
    d=json.loads(l); print(round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), '%.4g'%d['value'])
"; done
python -c "
import json,csv,glob
d=json.loads(open('$OUT/trace_c4.json').read().strip().splitlines()[-1])
f=glob.glob('$OUT/trace/**/c4_kernel_stats.csv', recursive=True) or glob.glob('$OUT/trace/*kernel_stats.csv')
for r in csv.DictReader(open(f[0])):
    if 'simulate_kernel' in r['Name']: print('rocprof avg us', float(r['AverageNs'])/1e3, 'calls', r['Calls'])
print('bench kernel_ms', d['roofline']['kernel_ms'], 'ms_per_step', d['ms_per_step'])
"

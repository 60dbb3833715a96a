# round 6: progress-based wave priorities (s_setprio 3 -> 0 over the frames: the waves a SIMD's
# oldest-first arbiter let run ahead yield to the ones behind) against the committed build
# (tools/_ab/lib_nofair.so), alternated on one box; the GPU suite first
export TMPDIR=/tmp
OUT=gpurun_out/r06r
mkdir -p $OUT
LIB=topotrafficrl_amd/lib/libttrl_mi355x.so
cp $LIB /tmp/lib_new.so || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for c in 4 2 3 5; do
    cp /tmp/lib_new.so $LIB && timeout -k 10 200 python bench.py --config $c --no-cpu-baseline >> $OUT/new_c$c.json 2>> $OUT/err || exit $?
    cp tools/_ab/lib_nofair.so $LIB && timeout -k 10 200 python bench.py --config $c --no-cpu-baseline >> $OUT/prev_c$c.json 2>> $OUT/err || exit $?
  done
done
for r in 1 2; do
  cp /tmp/lib_new.so $LIB && timeout -k 10 200 python bench.py --config 6 --no-cpu-baseline --steps 200 >> $OUT/new_c6.json 2>> $OUT/err || exit $?
  cp tools/_ab/lib_nofair.so $LIB && timeout -k 10 200 python bench.py --config 6 --no-cpu-baseline --steps 200 >> $OUT/prev_c6.json 2>> $OUT/err || exit $?
done
cp /tmp/lib_new.so $LIB
for f in $OUT/new_c*.json $OUT/prev_c*.json; do echo $f; python -c "
import json
for l in open('$f'):
    d=json.loads(l); print(round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), '%.4g'%d['value'])
"; done
mkdir -p $OUT/placement && timeout -k 10 200 python -u tools/placement.py $OUT/placement > $OUT/placement/summary.txt 2>&1 || exit $?

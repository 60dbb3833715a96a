# round 6: balanced intersection workgroups (the k-th heaviest env beside the k-th lightest): ix GPU
# tests, then config 6 against the previous build (tools/_ab/lib_prev.so) and envs paired by rank
# (heaviest with the next heaviest, tools/_ab/lib_sorted.so), alternated on one box
export TMPDIR=/tmp
OUT=gpurun_out/r06m
mkdir -p $OUT
LIB=topotrafficrl_amd/lib/libttrl_mi355x.so
cp $LIB /tmp/lib_new.so || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_ix_env.py tests/test_ops.py tests/test_gpu_ix.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  cp /tmp/lib_new.so $LIB && timeout -k 10 200 python bench.py --config 6 --no-cpu-baseline --steps 200 >> $OUT/new.json 2>> $OUT/err || exit $?
  cp tools/_ab/lib_prev.so $LIB && timeout -k 10 200 python bench.py --config 6 --no-cpu-baseline --steps 200 >> $OUT/prev.json 2>> $OUT/err || exit $?
  cp tools/_ab/lib_sorted.so $LIB && timeout -k 10 200 python bench.py --config 6 --no-cpu-baseline --steps 200 >> $OUT/sorted.json 2>> $OUT/err || exit $?
done
cp /tmp/lib_new.so $LIB
for f in $OUT/new.json $OUT/prev.json $OUT/sorted.json; do echo $f; python -c "
import json
for l in open('$f'):
    d=json.loads(l); print(round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), '%.4g'%d['value'])
"; done

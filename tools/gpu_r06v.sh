# round 6: rank-aware progress priorities (the SIMD's two oldest waves -- HW_ID's wave slot is the
# dispatch rank -- demote one frame before the two youngest at each quarter; source kept as
# tools/_ab/rankshift.hip, built as tools/_ab/lib_rankshift.so) against the quarter bins (the in-tree,
# profiled r06y build), alternated on one box
export TMPDIR=/tmp
OUT=gpurun_out/r06v
mkdir -p $OUT
LIB=topotrafficrl_amd/lib/libttrl_mi355x.so
cp $LIB /tmp/lib_quarters.so || exit 1
cp tools/_ab/lib_rankshift.so $LIB || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_env.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.txt 2>&1
rc=$?; cp /tmp/lib_quarters.so $LIB; echo "tests rc=$rc"; tail -2 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for c in 4 2 5; do
    cp tools/_ab/lib_rankshift.so $LIB && timeout -k 10 200 python bench.py --config $c --no-cpu-baseline >> $OUT/rankshift_c$c.json 2>> $OUT/err || exit $?
    cp /tmp/lib_quarters.so $LIB && timeout -k 10 200 python bench.py --config $c --no-cpu-baseline >> $OUT/quarters_c$c.json 2>> $OUT/err || exit $?
  done
done
cp /tmp/lib_quarters.so $LIB
for f in $OUT/*_c*.json; do echo $f; python -c "
import json
for l in open('$f'):
    d=json.loads(l); print(round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), '%.4g'%d['value'])
"; done

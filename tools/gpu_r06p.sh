# round 6: config 6 with every simulate instance at a 3-wave register budget (-DTTRL_SIM_WAVES=3:
# the step and the warm-ups at <= 168 VGPRs, so warm-up waves fit beside the step's two per SIMD
# instead of displacing its workgroups) against the committed build, alternated on one box
export TMPDIR=/tmp
OUT=gpurun_out/r06p
mkdir -p $OUT
LIB=topotrafficrl_amd/lib/libttrl_mi355x.so
cp $LIB /tmp/lib_cur.so || exit 1
for r in 1 2 3; do
  cp /tmp/lib_cur.so $LIB && timeout -k 10 200 python bench.py --config 6 --no-cpu-baseline --steps 200 >> $OUT/cur.json 2>> $OUT/err || exit $?
  cp tools/_ab/lib_w3.so $LIB && timeout -k 10 200 python bench.py --config 6 --no-cpu-baseline --steps 200 >> $OUT/w3.json 2>> $OUT/err || exit $?
done
cp /tmp/lib_cur.so $LIB
for f in $OUT/cur.json $OUT/w3.json; do echo $f; python -c "
import json
for l in open('$f'):
    d=json.loads(l); print(round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), '%.4g'%d['value'])
"; done

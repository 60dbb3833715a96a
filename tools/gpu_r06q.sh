# round 6: config 6's bimodal step time (0.49 or 0.595 ms from run to run of the same build): runs
# with HIP's default 4 hardware queues per process against 8 (GPU_MAX_HW_QUEUES), alternated, and the
# 3-wave-budget variant with 8 queues
export TMPDIR=/tmp
OUT=gpurun_out/r06q
mkdir -p $OUT
LIB=topotrafficrl_amd/lib/libttrl_mi355x.so
cp $LIB /tmp/lib_cur.so || exit 1
for r in 1 2 3 4 5; do
  GPU_MAX_HW_QUEUES=4 timeout -k 10 200 python bench.py --config 6 --no-cpu-baseline --steps 200 >> $OUT/q4.json 2>> $OUT/err || exit $?
  GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python bench.py --config 6 --no-cpu-baseline --steps 200 >> $OUT/q8.json 2>> $OUT/err || exit $?
done
for r in 1 2 3; do
  cp tools/_ab/lib_w3.so $LIB && GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python bench.py --config 6 --no-cpu-baseline --steps 200 >> $OUT/w3_q8.json 2>> $OUT/err || exit $?
  cp /tmp/lib_cur.so $LIB
done
cp /tmp/lib_cur.so $LIB
for f in $OUT/q4.json $OUT/q8.json $OUT/w3_q8.json; do echo $f; python -c "
import json
for l in open('$f'):
    d=json.loads(l); print(round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), '%.4g'%d['value'])
"; done

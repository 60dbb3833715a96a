# round 6: the progress priorities in end-weighted bins (3 until the last three frames, then 2, 1, 0;
# straight <= 64-slot instances only) against quarters on every instance (tools/_ab/lib_fairq.so) and
# no priorities (lib_nofair.so) for configs 4, 2, 5, 3; config 6 with the bins also on the road
# network (lib_fairgr.so) against without; alternated on one box
export TMPDIR=/tmp
OUT=gpurun_out/r06s
mkdir -p $OUT
LIB=topotrafficrl_amd/lib/libttrl_mi355x.so
cp $LIB /tmp/lib_new.so || exit 1
for r in 1 2; do
  for c in 4 2 5 3; do
    for v in new fairq nofair; do
      if [ $v = new ]; then cp /tmp/lib_new.so $LIB; else cp tools/_ab/lib_$v.so $LIB; fi
      timeout -k 10 200 python bench.py --config $c --no-cpu-baseline >> $OUT/${v}_c$c.json 2>> $OUT/err || exit $?
    done
  done
done
for r in 1 2 3; do
  cp /tmp/lib_new.so $LIB && timeout -k 10 200 python bench.py --config 6 --no-cpu-baseline --steps 200 >> $OUT/new_c6.json 2>> $OUT/err || exit $?
  cp tools/_ab/lib_fairgr.so $LIB && timeout -k 10 200 python bench.py --config 6 --no-cpu-baseline --steps 200 >> $OUT/fairgr_c6.json 2>> $OUT/err || exit $?
done
cp /tmp/lib_new.so $LIB
for f in $OUT/*_c*.json; do echo $f; python -c "
import json
for l in open('$f'):
    d=json.loads(l); print(round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), '%.4g'%d['value'])
"; done

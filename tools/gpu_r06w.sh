# round 6: config 3 with the progress priorities on its second round of workgroups only (blocks in the
# upper half of the grid; source kept as tools/_ab/round2.hip, built as tools/_ab/lib_round2.so)
# against the in-tree build (no priorities at 128 slots), alternated on one box
export TMPDIR=/tmp
OUT=gpurun_out/r06w
mkdir -p $OUT
LIB=topotrafficrl_amd/lib/libttrl_mi355x.so
cp $LIB /tmp/lib_cur.so || exit 1
for r in 1 2 3; do
  cp tools/_ab/lib_round2.so $LIB && timeout -k 10 200 python bench.py --config 3 --no-cpu-baseline >> $OUT/round2_c3.json 2>> $OUT/err || exit $?
  cp /tmp/lib_cur.so $LIB && timeout -k 10 200 python bench.py --config 3 --no-cpu-baseline >> $OUT/cur_c3.json 2>> $OUT/err || exit $?
done
cp /tmp/lib_cur.so $LIB
for f in $OUT/*_c*.json; do echo $f; python -c "
import json
for l in open('$f'):
    d=json.loads(l); print(round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), '%.4g'%d['value'])
"; done

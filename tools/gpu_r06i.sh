# round 6: config 3's fused grid write-out, plain stores (product build) vs nontemporal stores
# (tools/_ab/lib_gridnt.so, -DTTRL_GRID_NT_STORES=1) vs the two-launch step, alternated in one box
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out
cd $GRAFT_REPO_ROOT || exit 1
mkdir -p $OUT/r06i
LIB=topotrafficrl_amd/lib/libttrl_mi355x.so
cp $LIB /tmp/lib_plain.so || exit 1
timeout -k 10 300 python -u -m pytest tests/test_ops.py tests/test_gpu_env.py -m gpu -x -q --timeout 120 --timeout-method thread -k "grid or fused_step_tail" > $OUT/r06i/tests.txt 2>&1
rc=$?
echo "tests rc=$rc"
[ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  cp /tmp/lib_plain.so $LIB && timeout -k 10 200 python bench.py --config 3 --no-cpu-baseline --steps 50 >> $OUT/r06i/plain.json 2>> $OUT/r06i/err || exit $?
  cp tools/_ab/lib_gridnt.so $LIB && timeout -k 10 200 python bench.py --config 3 --no-cpu-baseline --steps 50 >> $OUT/r06i/nt.json 2>> $OUT/r06i/err || exit $?
  TTRL_FUSE_GRID=0 timeout -k 10 200 python bench.py --config 3 --no-cpu-baseline --steps 50 >> $OUT/r06i/twolaunch.json 2>> $OUT/r06i/err || exit $?
done
cp /tmp/lib_plain.so $LIB
echo done

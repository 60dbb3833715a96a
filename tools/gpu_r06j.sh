# round 6: the NS = 128 instances' tie-path masks and frame-0 action address laundered (32 -> 8 B/lane
# scratch; fused grid 44 -> 20): GPU parity of the 128-slot paths, and config 3 against the previous
# build (tools/_ab/lib_gridnt.so) and the two-launch step, alternated in one box
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out
cd $GRAFT_REPO_ROOT || exit 1
mkdir -p $OUT/r06j
LIB=topotrafficrl_amd/lib/libttrl_mi355x.so
cp $LIB /tmp/lib_new.so || exit 1
timeout -k 10 500 python -u -m pytest tests/test_ops.py tests/test_gpu_env.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/r06j/tests.txt 2>&1
rc=$?
echo "tests rc=$rc"
[ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  cp /tmp/lib_new.so $LIB && timeout -k 10 200 python bench.py --config 3 --no-cpu-baseline --steps 50 >> $OUT/r06j/new.json 2>> $OUT/r06j/err || exit $?
  TTRL_FUSE_GRID=0 timeout -k 10 200 python bench.py --config 3 --no-cpu-baseline --steps 50 >> $OUT/r06j/new_twolaunch.json 2>> $OUT/r06j/err || exit $?
  cp tools/_ab/lib_gridnt.so $LIB && timeout -k 10 200 python bench.py --config 3 --no-cpu-baseline --steps 50 >> $OUT/r06j/prev.json 2>> $OUT/r06j/err || exit $?
done
cp /tmp/lib_new.so $LIB
echo done

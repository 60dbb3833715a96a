# round 6: config 3's OccupancyGrid written by the step launch (ttrl_env_step_grid): tests, the
# full-size grid parity, and config-3 bench lines fused vs two launches in one box
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out
cd $GRAFT_REPO_ROOT || exit 1
mkdir -p $OUT/r06g
timeout -k 10 400 python -u -m pytest tests/test_ops.py tests/test_gpu_env.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/r06g/tests.txt 2>&1
rc=$?
echo "tests rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread -k occupancy > $OUT/r06g/fullsize.txt 2>&1
rc=$?
echo "fullsize rc=$rc"
[ $rc -eq 0 ] || exit $rc
for v in 1 0 1 0; do
  TTRL_FUSE_GRID=$v timeout -k 10 200 python bench.py --config 3 --no-cpu-baseline --steps 50 >> $OUT/r06g/bench_c3_fuse$v.json 2>> $OUT/r06g/bench_c3.err || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r06g -o c3trace -- python3 bench.py --config 3 --no-cpu-baseline --steps 20 > $OUT/r06g/c3trace.log 2>&1 || exit $?
echo done

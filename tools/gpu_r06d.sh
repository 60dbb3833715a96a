# round 6: the fused intersection tail (ttrl_ix_env_step): its GPU tests, then config 6 fused and unfused
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out
cd $GRAFT_REPO_ROOT || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_ix_env.py tests/test_ops.py tests/test_gpu_ix.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/r06d_ix_tests.txt 2>&1
rc=$?
echo "ix tests rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config 6 --no-cpu-baseline > $OUT/r06d_bench_c6.json 2> $OUT/r06d_bench_c6.err || exit $?
TTRL_IX_FUSE_TAIL=0 timeout -k 10 300 python bench.py --config 6 --no-cpu-baseline > $OUT/r06d_bench_c6_unfused.json 2> $OUT/r06d_bench_c6_unfused.err || exit $?
timeout -k 10 300 python bench.py --config 6 --no-cpu-baseline --steps 200 > $OUT/r06d_bench_c6_200.json 2> $OUT/r06d_bench_c6_200.err || exit $?
echo done

# round 6: the r05e 16-slot / four-envs-per-wave divergence reproduced on its own tree (commit
# 2947fbf, extracted under tools/_bisect/r05e) with and without the list-length fix, then the GPU
# suite and the default bench line on the current tree
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out
B=$GRAFT_REPO_ROOT/tools/_bisect/r05e
cd $B || exit 1
for v in buggy fixed; do
  cp lib_$v/*.so topotrafficrl_amd/lib/ || exit 1
  timeout -k 10 240 python tools/ix_ns16.py 30 > $OUT/r06a_ns16_$v.txt 2>&1 || exit $?
  timeout -k 10 300 python -u -m pytest tests/test_gpu_ix_env.py -m gpu -q -k "slot_classes or overlapped" --timeout 120 --timeout-method thread > $OUT/r06a_ix_tests_$v.txt 2>&1
  rc=$?
  echo "$v tests rc=$rc"
  [ $rc -le 1 ] || exit $rc
done
cd $GRAFT_REPO_ROOT || exit 1
TTRL_PARITY_LOG=$OUT/r06a_parity.json timeout -k 10 600 python -u -m pytest tests -m gpu -q -rs --timeout 120 --timeout-method thread > $OUT/r06a_gpu_tests.txt 2>&1
rc=$?
echo "suite rc=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/r06a_bench.json 2> $OUT/r06a_bench.err || exit $?
echo done

# round 5, final tree: the GPU suite, smoke, the default bench line (config 4 with its CPU baselines)
export TMPDIR=/tmp
OUT=gpurun_out/r05final
mkdir -p $OUT
TTRL_PARITY_LOG=$OUT/parity.json timeout -k 10 600 python -u -m pytest tests -m gpu -q -rs --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1 || exit $?
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?

# round 6, fresh container rebuild: the whole GPU suite, smoke, the default bench line and config 6
export TMPDIR=/tmp
OUT=gpurun_out/r06k
mkdir -p $OUT
sha256sum topotrafficrl_amd/lib/*.so > $OUT/sha.txt
TTRL_PARITY_LOG=$OUT/parity.json timeout -k 10 700 python -u -m pytest tests -m gpu -q -rs --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/gpu_tests.txt; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1 || exit $?
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
cat $OUT/bench.json
timeout -k 10 300 python bench.py --config 6 --no-cpu-baseline --steps 200 > $OUT/bench_c6_200.json 2> $OUT/bench_c6.err || exit $?
cat $OUT/bench_c6_200.json

# round 5: the road-network instance's projection / regulation / steering changes: A/B, phases, GPU suite, config 6
export TMPDIR=/tmp
OUT=gpurun_out/r05o
mkdir -p $OUT
IX=1 timeout -k 10 300 python tools/variants.py run f64 f32 > $OUT/ix_ab.txt 2>&1 || exit $?
timeout -k 10 200 python tools/phases.py f64 15 --ix > $OUT/phases_ix_f64.txt 2>&1 || exit $?
TTRL_PARITY_LOG=$OUT/parity.json timeout -k 10 600 python -u -m pytest tests -m gpu -q -rs --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --config 6 --no-cpu-baseline > $OUT/bench_c6.json 2> $OUT/bench_c6.err || exit $?

# round 5: the straight instance's overflow sweep inlined again (no scratch on the headline launch):
# A/B against the committed kernel, the GPU suite, bench lines
export TMPDIR=/tmp
OUT=gpurun_out/r05y
mkdir -p $OUT
timeout -k 10 200 python tools/variants.py run f64 f32 > $OUT/ab_c4.txt 2>&1 || exit $?
N=32 E=4096 timeout -k 10 200 python tools/variants.py run f64 > $OUT/ab_c2.txt 2>&1 || exit $?
TTRL_PARITY_LOG=$OUT/parity.json timeout -k 10 600 python -u -m pytest tests -m gpu -q -rs --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || exit $?
timeout -k 10 300 python bench.py --config 2 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit $?
timeout -k 10 300 python bench.py --config 6 --no-cpu-baseline > $OUT/bench_c6.json 2> $OUT/bench_c6.err || exit $?

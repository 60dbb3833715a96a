# round 5: regulation pairs in chunks (no serial fallback past RQ_PAIRS), SAT proofs in one round:
# intersection A/B and phases, the GPU suite, bench lines for configs 6, 4 and 2
export TMPDIR=/tmp
OUT=gpurun_out/r05q
mkdir -p $OUT
IX=1 timeout -k 10 300 python tools/variants.py run f64 f32 > $OUT/ix_ab.txt 2>&1 || exit $?
timeout -k 10 200 python tools/phases.py f64 15 --ix > $OUT/phases_ix_f64.txt 2>&1 || exit $?
TTRL_PARITY_LOG=$OUT/parity.json timeout -k 10 600 python -u -m pytest tests -m gpu -q -rs --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --config 6 --no-cpu-baseline > $OUT/bench_c6.json 2> $OUT/bench_c6.err || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_c4.json 2> $OUT/bench_c4.err || exit $?
timeout -k 10 300 python bench.py --config 2 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit $?

# round 5: the GPU suite and the bench lines on the current build
export TMPDIR=/tmp
TTRL_PARITY_LOG=gpurun_out/r05f_parity.json timeout -k 10 600 python -u -m pytest tests -m gpu -q -rs --timeout 300 --timeout-method thread > gpurun_out/r05f_gpu_tests.txt 2>&1
rc=$?
echo "tests rc=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --config 6 --no-cpu-baseline > gpurun_out/r05f_bench_c6.json 2> gpurun_out/r05f_bench_c6.err || exit $?
timeout -k 10 300 python bench.py --config 2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05f_bench_c2.json 2> gpurun_out/r05f_bench_c2.err || exit $?
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r05f_bench.json 2> gpurun_out/r05f_bench.err

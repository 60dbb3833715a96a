# round 5: the mixed intersection dispatch measured, the GPU suite, the bench lines of configs 2, 6
# and 4, then diagnostics (head vs working-tree A/B, the headline's phases and instruction mix)
export TMPDIR=/tmp
timeout -k 10 200 python tools/ix_ns16.py > gpurun_out/r05e_ns16.txt 2>&1
rc=$?
echo "ns16 rc=$rc"
[ $rc -le 1 ] || exit $rc
TTRL_PARITY_LOG=gpurun_out/r05e_parity.json timeout -k 10 600 python -u -m pytest tests -m gpu -q -rs --timeout 300 --timeout-method thread > gpurun_out/r05e_gpu_tests.txt 2>&1
rc=$?
echo "tests rc=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --config 2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05e_bench_c2.json 2> gpurun_out/r05e_bench_c2.err || exit $?
timeout -k 10 300 python bench.py --config 6 --no-cpu-baseline > gpurun_out/r05e_bench_c6.json 2> gpurun_out/r05e_bench_c6.err || exit $?
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r05e_bench.json 2> gpurun_out/r05e_bench.err || exit $?
timeout -k 10 300 python tools/variants.py run f64 f32 > gpurun_out/r05e_variants.txt 2>&1 || exit $?
timeout -k 10 200 python tools/phases.py f64 > gpurun_out/r05e_phases_f64.txt 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d gpurun_out/r05e_insts -o insts -- python3 tools/insts.py > gpurun_out/r05e_insts.log 2>&1 || exit $?
python3 tools/insts.py --report gpurun_out/r05e_insts/insts_counter_collection.csv > gpurun_out/r05e_insts.txt 2>&1

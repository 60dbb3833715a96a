# round 6: fused-tail tests + config 6; the headline reconciliation: round-4 (ec952d4), round-5
# (5e3157c) and current builds of the fused launch timed and profiled in one process each
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out
cd $GRAFT_REPO_ROOT || exit 1
mkdir -p $OUT/r06f
timeout -k 10 400 python -u -m pytest tests/test_gpu_ix_env.py tests/test_ops.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/r06f/ix_tests.txt 2>&1
rc=$?
echo "ix tests rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config 6 --no-cpu-baseline --steps 200 > $OUT/r06f/bench_c6_200.json 2> $OUT/r06f/bench_c6_200.err || exit $?
export REV_VARIANTS="r04=ec952d4;r05=5e3157c"
timeout -k 10 300 python tools/variants.py run f64 > $OUT/r06f/ab.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r06f -o abtrace -- python3 tools/variants.py run f64 > $OUT/r06f/abtrace.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/r06f -o absq -- python3 tools/variants.py run f64 > $OUT/r06f/absq.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/r06f -o abgrbm -- python3 tools/variants.py run f64 > $OUT/r06f/abgrbm.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/r06f -o abfetch -- python3 tools/variants.py run f64 > $OUT/r06f/abfetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/r06f -o abwrite -- python3 tools/variants.py run f64 > $OUT/r06f/abwrite.log 2>&1 || exit $?
K=simulate_kernelIdLi64ELi1ELi0E
for f in abtrace_kernel_trace absq_counter_collection abgrbm_counter_collection abfetch_counter_collection abwrite_counter_collection; do
  python3 tools/ab_trace.py $OUT/r06f/$f.csv $K 20 cur,r04,r05 >> $OUT/r06f/ab_summary.txt 2>&1
done
echo done

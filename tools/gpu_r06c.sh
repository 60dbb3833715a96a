# round 6: config 6 kernel trace on the fused build
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out
cd $GRAFT_REPO_ROOT || exit 1
mkdir -p $OUT/r06e
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r06e -o c6 -- python3 bench.py --config 6 --steps 60 --warmup 10 --no-cpu-baseline > $OUT/r06e/bench_c6.json 2> $OUT/r06e/c6_trace.err || exit $?
python3 tools/trace_durations.py $OUT/r06e/c6_kernel_trace.csv simulate_ix_kernel > $OUT/r06e/c6_durations.txt 2>&1
echo done

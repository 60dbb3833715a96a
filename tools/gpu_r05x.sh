# round 5: config 6 on the committed build (spare resets one workgroup per row), for comparison
export TMPDIR=/tmp
OUT=gpurun_out/r05x
mkdir -p $OUT
timeout -k 10 300 python bench.py --config 6 --no-cpu-baseline > $OUT/bench_c6.json 2> $OUT/bench_c6.err || exit $?
timeout -k 10 300 python bench.py --config 6 --steps 200 --warmup 10 --no-cpu-baseline > $OUT/bench_c6_200.json 2> $OUT/bench_c6_200.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o c6 -- python3 bench.py --config 6 --steps 40 --warmup 10 --no-cpu-baseline > $OUT/bench_c6_trace.json 2> $OUT/c6_trace.err || exit $?

# round 5, final tree: the remaining bench lines (configs 3 and 5) and the 2-rank shared-GPU rehearsal
export TMPDIR=/tmp
OUT=gpurun_out/r05extra
mkdir -p $OUT
timeout -k 10 300 python bench.py --config 3 --no-cpu-baseline > $OUT/bench_c3.json 2> $OUT/bench_c3.err || exit $?
timeout -k 10 300 python bench.py --config 5 --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.err || exit $?
TTRL_BENCH_SHARED_GPU=1 timeout -k 10 400 python bench.py --gpus 2 --no-cpu-baseline > $OUT/bench2.json 2> $OUT/bench2.err || exit $?

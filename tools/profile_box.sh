#!/bin/bash
# Run ON the GPU box (gpurun): kernel-trace stats + separate PMC passes for the bench workload.
# Outputs under gpurun_out/prof_$TAG; summarise with tools/profile_summary.py.
set -e
TAG=${TAG:-r01}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
for DT in f64 f32; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o trace_$DT -- \
    python3 bench.py --steps 20 --warmup 3 --dtype $DT --no-cpu-baseline > $OUT/bench_trace_$DT.json 2> $OUT/trace_$DT.err
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT -o fetch_$DT -- \
    python3 bench.py --steps 5 --warmup 1 --dtype $DT --no-cpu-baseline > /dev/null 2> $OUT/fetch_$DT.err
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT -o write_$DT -- \
    python3 bench.py --steps 5 --warmup 1 --dtype $DT --no-cpu-baseline > /dev/null 2> $OUT/write_$DT.err
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $OUT -o sq_$DT -- \
    python3 bench.py --steps 5 --warmup 1 --dtype $DT --no-cpu-baseline > /dev/null 2> $OUT/sq_$DT.err
  timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT -o grbm_$DT -- \
    python3 bench.py --steps 5 --warmup 1 --dtype $DT --no-cpu-baseline > /dev/null 2> $OUT/grbm_$DT.err
done
echo profile done
# config 3 (4096 x 128, OccupancyGrid 7x32x32): kernel stats + HBM traffic of the simulate and grid launches
if [ "${CONFIG3:-1}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o trace_c3 -- \
    python3 bench.py --config 3 --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_trace_c3.json 2> $OUT/trace_c3.err
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT -o fetch_c3 -- \
    python3 bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/fetch_c3.err
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT -o write_c3 -- \
    python3 bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/write_c3.err
fi
echo profile c3 done

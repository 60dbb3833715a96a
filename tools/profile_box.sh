#!/bin/bash
# Run ON the GPU box (gpurun): for every bench configuration in $RUNS ("config:dtype" pairs), a
# kernel-trace stats run of bench.py and separate PMC passes (FETCH_SIZE, WRITE_SIZE, the SQ
# instruction mix, the SQ LDS / wait counters, GRBM for the clock), one counter group per run as
# MI355X_MICROARCH.md prescribes.  Outputs under gpurun_out/prof_$TAG; summarise with
# tools/profile_summary.py $TAG (which writes profiles/pmc_traffic.json for this build).
set -e
TAG=${TAG:-r01}
RUNS=${RUNS:-"4:f64 4:f32 3:f64 2:f64 5:f64 6:f64"}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
for R in $RUNS; do
  C=${R%%:*}; DT=${R##*:}; N=c${C}_${DT}
  STEPS="--steps 20 --warmup 3"; PSTEPS="--steps 5 --warmup 1"
  if [ "$C" = "6" ]; then STEPS="--steps 40 --warmup 10"; PSTEPS="--steps 10 --warmup 10"; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o trace_$N -- \
    python3 bench.py --config $C --dtype $DT $STEPS --no-cpu-baseline > $OUT/bench_trace_$N.json 2> $OUT/trace_$N.err
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT -o fetch_$N -- \
    python3 bench.py --config $C --dtype $DT $PSTEPS --no-cpu-baseline > /dev/null 2> $OUT/fetch_$N.err
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT -o write_$N -- \
    python3 bench.py --config $C --dtype $DT $PSTEPS --no-cpu-baseline > /dev/null 2> $OUT/write_$N.err
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $OUT -o sq_$N -- \
    python3 bench.py --config $C --dtype $DT $PSTEPS --no-cpu-baseline > /dev/null 2> $OUT/sq_$N.err
  timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_INSTS_SMEM SQ_INST_CYCLES_SALU --output-format csv -d $OUT -o sq2_$N -- \
    python3 bench.py --config $C --dtype $DT $PSTEPS --no-cpu-baseline > /dev/null 2> $OUT/sq2_$N.err
  timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT -o grbm_$N -- \
    python3 bench.py --config $C --dtype $DT $PSTEPS --no-cpu-baseline > /dev/null 2> $OUT/grbm_$N.err
  echo "profile $N done"
done

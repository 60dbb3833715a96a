# round 5: config 6 attribution -- per-phase cycles of the intersection instance, and the SQ
# activity counters (scalar / LDS / any instruction issue) of config 6's and config 4's launches
export TMPDIR=/tmp
OUT=gpurun_out/r05h
mkdir -p $OUT
timeout -k 10 200 python tools/phases.py f64 15 --ix > $OUT/phases_ix_f64.txt 2>&1 || exit $?
timeout -k 10 200 python tools/phases.py f64 > $OUT/phases_f64.txt 2>&1 || exit $?
for C in 6 4; do
  P="--steps 5 --warmup 1"; [ $C = 6 ] && P="--steps 10 --warmup 10"
  timeout -s KILL 200 rocprofv3 --pmc SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS SQ_LDS_ADDR_CONFLICT SQ_WAVE_CYCLES SQ_WAVES --output-format csv -d $OUT -o sq3_c$C -- \
    python3 bench.py --config $C $P --no-cpu-baseline > /dev/null 2> $OUT/sq3_c$C.err || exit $?
  echo "sq3 c$C done"
done

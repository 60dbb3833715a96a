# round 5: intersection phases over in-loop scenes; config 2 (4096 x 32) with one env per wave
export TMPDIR=/tmp
OUT=gpurun_out/r05i
mkdir -p $OUT
timeout -k 10 200 python tools/phases.py f64 15 --ix > $OUT/phases_ix_f64.txt 2>&1 || exit $?
EDIT_VARIANTS=ns32x1 N=32 E=4096 timeout -k 10 200 python tools/variants.py run f64 f32 > $OUT/ns32x1.txt 2>&1 || exit $?

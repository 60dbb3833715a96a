# round 5: A/B of the committed kernel against the working tree (highway 64 / 32 slots, intersection),
# intersection phases with the regulation's fallback counts
export TMPDIR=/tmp
OUT=gpurun_out/r05p
mkdir -p $OUT
timeout -k 10 200 python tools/variants.py run f64 f32 > $OUT/ab_c4.txt 2>&1 || exit $?
N=32 E=4096 timeout -k 10 200 python tools/variants.py run f64 > $OUT/ab_c2.txt 2>&1 || exit $?
IX=1 timeout -k 10 300 python tools/variants.py run f64 f32 > $OUT/ix_ab.txt 2>&1 || exit $?
timeout -k 10 200 python tools/phases.py f64 15 --ix > $OUT/phases_ix_f64.txt 2>&1 || exit $?
timeout -k 10 200 python tools/phases.py f64 > $OUT/phases_f64.txt 2>&1 || exit $?

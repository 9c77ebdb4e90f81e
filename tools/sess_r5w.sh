#!/bin/bash
# Where the first BRECQ act phase's extra time goes: the full ResNet-18 W2A4 --bias_cal flow
# under tools/e2e_breakdown.py twice (the first process warms the box), the second with the
# per-iteration hook (setup / eager warm-up / capture / steady phases of every loop).
TAG=${1:-r5w}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
A="--arch resnet18 --n_bits_w 2 --n_bits_a 4 --weight 1.0 --bias_cal True --bias_ch_quant True"
SSQ_BREAKDOWN_HOOK=0 timeout -k 10 300 python tools/e2e_breakdown.py $A > $OUT/bd_${TAG}_cold.log 2>&1 || { echo "breakdown cold failed"; tail -5 $OUT/bd_${TAG}_cold.log; exit 1; }
grep "calibration finished\|brecq_loop #" $OUT/bd_${TAG}_cold.log | cut -c1-150
SSQ_BREAKDOWN_HOOK=1 timeout -k 10 300 python tools/e2e_breakdown.py $A > $OUT/bd_${TAG}_hook.log 2>&1 || { echo "breakdown hook failed"; tail -5 $OUT/bd_${TAG}_hook.log; exit 1; }
grep "calibration finished\|brecq_loop #\|brecq setup" $OUT/bd_${TAG}_hook.log | cut -c1-200
SSQ_BREAKDOWN_HOOK=0 timeout -k 10 300 python -m cProfile -o $OUT/bd_${TAG}.prof tools/e2e_breakdown.py $A > $OUT/bd_${TAG}_prof.log 2>&1 || { echo "cprofile failed"; tail -5 $OUT/bd_${TAG}_prof.log; exit 1; }
grep "calibration finished\|brecq_loop #" $OUT/bd_${TAG}_prof.log | cut -c1-150
python -c "import pstats; pstats.Stats('$OUT/bd_${TAG}.prof').sort_stats('cumtime').print_stats(45)" > $OUT/bd_${TAG}_prof_cum.txt 2>&1
python -c "import pstats; pstats.Stats('$OUT/bd_${TAG}.prof').sort_stats('tottime').print_stats(30)" > $OUT/bd_${TAG}_prof_tot.txt 2>&1
exit 0

#!/bin/bash
# cProfile of the full ResNet-18 W2A4 --bias_cal flow (second process on the box).
TAG=${1:-r5u}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
A="--arch resnet18 --n_bits_w 2 --n_bits_a 4 --weight 1.0 --bias_cal True --bias_ch_quant True"
SSQ_BREAKDOWN_HOOK=0 timeout -k 10 300 python tools/e2e_breakdown.py $A > $OUT/bd_${TAG}_cold.log 2>&1 || { echo "breakdown cold failed"; tail -5 $OUT/bd_${TAG}_cold.log; exit 1; }
grep "calibration finished" $OUT/bd_${TAG}_cold.log | cut -c1-120
SSQ_BREAKDOWN_HOOK=0 timeout -k 10 300 python -m cProfile -o $OUT/bd_${TAG}.prof tools/e2e_breakdown.py $A > $OUT/bd_${TAG}_prof.log 2>&1 || { echo "cprofile failed"; tail -5 $OUT/bd_${TAG}_prof.log; exit 1; }
grep "calibration finished" $OUT/bd_${TAG}_prof.log | cut -c1-120
exit 0

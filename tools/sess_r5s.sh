#!/bin/bash
# r5s: the GPU suite with the frozen-weight GEMM forward (BRECQ act phase, layer3/4 convs),
# the act phase's anatomy, and the end-to-end per-call breakdown with the route on / off.
TAG=${1:-r5s}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
cd $R
bash tools/sess_tests.sh $TAG
rc=$?
[ $rc -ne 0 ] && exit $rc
bash tools/act_anatomy.sh $TAG || exit 1
grep -- "---" $OUT/act_anatomy_$TAG.txt | head -8
A="--arch resnet18 --n_bits_w 2 --n_bits_a 4 --weight 1.0 --bias_cal True --bias_ch_quant True"
for V in 1 0 1; do
  SSQ_FROZEN_FWD_GEMM=$V SSQ_BREAKDOWN_HOOK=0 timeout -k 10 300 python tools/e2e_breakdown.py $A > $OUT/bd_${TAG}_$V.log 2>&1 || { echo "breakdown $V failed"; tail -5 $OUT/bd_${TAG}_$V.log; exit 1; }
  echo "SSQ_FROZEN_FWD_GEMM=$V $(grep 'calibration finished' $OUT/bd_${TAG}_$V.log | cut -c1-90) brecq_loop ms: $(grep 'brecq_loop #' $OUT/bd_${TAG}_$V.log | awk '{print $4}' | tr '\n' ' ')"
done

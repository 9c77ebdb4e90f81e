#!/bin/bash
# End-to-end wall time at the tree's kernels: the full ResNet-18 W2A4 --bias_cal flow
# unprofiled, then the act phase's per-iteration anatomy (tools/act_anatomy.sh).
# Usage (via gpurun): bash tools/sess_e2e.sh TAG [extra env assignments for the e2e run]
TAG=${1:-e2e}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 600 python main_imagenet.py --arch resnet18 --n_bits_w 2 --n_bits_a 4 --weight 1.0 --bias_cal True --bias_ch_quant True > $OUT/e2e_$TAG.log 2>&1 || { echo "e2e failed"; tail -20 $OUT/e2e_$TAG.log; exit 1; }
grep "calibration finished" $OUT/e2e_$TAG.log | cut -c1-160
bash tools/act_anatomy.sh $TAG || exit 1
grep -- "---" $OUT/act_anatomy_$TAG.txt | head -12
exit 0

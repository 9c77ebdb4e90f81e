#!/bin/bash
# Per-call wall times of the full ResNet-18 W2A4 --bias_cal flow (tools/e2e_breakdown.py, no
# per-iteration hook), at the defaults and with r5's loop changes off one at a time.
TAG=${1:-bd}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
A="--arch resnet18 --n_bits_w 2 --n_bits_a 4 --weight 1.0 --bias_cal True --bias_ch_quant True"
for V in "default" "SSQ_FUSE_FC=0" "SSQ_BRECQ_ROWS=0" "SSQ_BRECQ_CHUNK=1"; do
  if [ "$V" = default ]; then E=""; else E="$V"; fi
  env $E SSQ_BREAKDOWN_HOOK=0 timeout -k 10 300 python tools/e2e_breakdown.py $A > $OUT/bd_${TAG}_${V}.log 2>&1 || { echo "breakdown $V failed"; tail -5 $OUT/bd_${TAG}_${V}.log; exit 1; }
  echo "== $V"; grep "^\[breakdown\] \(total\|  \|[a-z_]* *[0-9]* calls\)" $OUT/bd_${TAG}_${V}.log | grep -v "#"
done

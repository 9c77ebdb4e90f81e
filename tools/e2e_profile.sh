#!/bin/bash
# Full README-default ResNet-18 W2A4 calibration under rocprofv3 (kernel stats only kept).
TAG=${1:-run}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 1100 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/e2eprof -o e2e -- python3 $R/main_imagenet.py --arch resnet18 --n_bits_w 2 --n_bits_a 4 --weight 1.0 --bias_cal True --bias_ch_quant True > $OUT/e2e_prof_$TAG.log 2>&1 || { echo "failed"; tail -20 $OUT/e2e_prof_$TAG.log; exit 1; }
cp $(find /tmp/e2eprof -name "*kernel_stats.csv" | head -1) $OUT/e2e_kernel_stats_$TAG.csv
grep "calibration finished" $OUT/e2e_prof_$TAG.log | cut -c1-200

#!/bin/bash
# Kernel trace of a short main_imagenet.py W2A4 bias_cal flow (50 shift iterations, 50 fc
# AdaRound iterations, 400 act-phase iterations per block) and the per-iteration anatomy of
# every recon segment (tools/trace_iter.py): the act phase's (BRECQ act-delta LSQ) launches.
TAG=${1:-run}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_act_$TAG -o act -- python3 $R/main_imagenet.py --arch resnet18 --n_bits_w 2 --n_bits_a 4 --weight 1.0 --bias_cal True --bias_ch_quant True --shift_iters 50 --iters_w 50 --iters_a 400 > $OUT/prof_act_$TAG.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof_act_$TAG.log; exit 1; }
KT=$(find $OUT/prof_act_$TAG -name "*kernel_trace.csv" | head -1)
MARKER=fin_tasks_kernel python3 $R/tools/trace_iter.py "$KT" full > $OUT/act_anatomy_$TAG.txt 2>&1
gzip -c "$KT" > $OUT/act_trace_$TAG.csv.gz
rm -f "$KT"
grep "calibration finished" $OUT/prof_act_$TAG.log | cut -c1-200

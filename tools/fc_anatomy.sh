#!/bin/bash
# The fc AdaRound loop (tools/fc_recon_rate.py) under rocprofv3 --kernel-trace: wall vs GPU
# busy per iteration (tools/trace_iter.py, iterations marked by the index copy).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
TAG=${1:-fc}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_fc_$TAG -o fc -- python3 $R/tools/fc_recon_rate.py > $OUT/prof_fc_$TAG.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof_fc_$TAG.log; exit 1; }
KT=$(find $OUT/prof_fc_$TAG -name "*kernel_trace.csv" | head -1)
MARKER=copyBuffer python3 $R/tools/trace_iter.py "$KT" > $OUT/fc_anatomy_$TAG.txt 2>&1
rm -f "$KT"
grep fc_adaround $OUT/prof_fc_$TAG.log

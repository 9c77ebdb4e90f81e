#!/bin/bash
# rocprofv3 kernel trace of tools/brecq_bench.py + per-iteration anatomy (tools/trace_iter.py)
TAG=${1:-run}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_brecq_$TAG -o brecq -- python3 $R/tools/brecq_bench.py > $OUT/prof_brecq_$TAG.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof_brecq_$TAG.log; exit 1; }
KT=$(find $OUT/prof_brecq_$TAG -name "*kernel_trace.csv" | head -1)
python3 $R/tools/trace_iter.py "$KT" > $OUT/brecq_anatomy_$TAG.txt 2>&1
tail -1 $OUT/prof_brecq_$TAG.log

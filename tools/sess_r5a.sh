#!/bin/bash
# r5a: GPU suite + smoke, then the launch-floor probe (tools/floor_probe.hip) plain and under
# rocprofv3 --kernel-trace.
TAG=${1:-r5a}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
bash tools/sess_tests.sh $TAG || exit $?
timeout -k 10 120 ./tools/floor_probe > $OUT/floor_probe_$TAG.json 2>&1 || { echo "floor probe failed"; tail -5 $OUT/floor_probe_$TAG.json; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/floorprof_$TAG -o fp -- $R/tools/floor_probe > $OUT/floor_probe_prof_$TAG.json 2>&1 || { echo "rocprof floor probe failed"; exit 1; }
KT=$(find $OUT/floorprof_$TAG -name "*kernel_trace.csv" | head -1)
[ -n "$KT" ] && python3 $R/tools/floor_summary.py "$KT" > $OUT/floor_trace_$TAG.txt 2>&1
[ -n "$KT" ] && rm -f "$KT"
exit 0
